#!/bin/bash
# Build libafivo_hip.so variants for scripts/ab.sh into ab/<name>/:
#   build_variant.sh <name> <git-rev|WORK> [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
src=/tmp/afh_variant_$name
rm -rf $src && mkdir -p $src/afivo-streamer_amd/csrc $src/include
if [ "$rev" = WORK ]; then
  cp afivo-streamer_amd/csrc/*.hip afivo-streamer_amd/csrc/*.h afivo-streamer_amd/csrc/Makefile $src/afivo-streamer_amd/csrc/
  cp include/*.h $src/include/
else
  for f in $(git ls-tree --name-only $rev afivo-streamer_amd/csrc/ include/); do git show $rev:$f > $src/$f; done
fi
make -s -C $src/afivo-streamer_amd/csrc -j8 HIPFLAGS_EXTRA="$*" >/dev/null
mkdir -p abv/$name && cp $src/afivo-streamer_amd/csrc/libafivo_hip.so abv/$name/
echo "abv/$name/libafivo_hip.so"
