"""The Fortran side of the drop-in boundary (fortran/m_afivo_hip.F90): one
bind(C) interface per entry point of include/afivo_hip.h, checked by name
both ways, and INTEGRATION.md's sharded-regrid snippet
(tests/fortran/regrid_rows.F90) compiled against the module with amdflang
(no GPU, no link)."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "afivo_hip.h")
MODULE = os.path.join(REPO, "afivo-streamer_amd", "fortran", "m_afivo_hip.F90")
SNIPPET = os.path.join(REPO, "tests", "fortran", "regrid_rows.F90")
FLANG = shutil.which("amdflang") or "/opt/rocm/llvm/bin/amdflang"


def header_symbols():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return set(re.findall(r"\b(afh_\w+)\s*\(", text))


def fortran_symbols():
    text = open(MODULE).read()
    return {"afh_" + s for s in re.findall(r'afh_pfx\s*//\s*"(\w+)"', text)}


def test_every_header_symbol_bound_in_fortran():
    h, f = header_symbols(), fortran_symbols()
    assert h - f == set(), "declared in the header, no bind(C) interface"
    assert f - h == set(), "bound in Fortran, not declared in the header"
    assert len(h) >= 76


@pytest.mark.skipif(not os.path.exists(FLANG), reason="amdflang not in the image")
def test_integration_snippet_compiles(tmp_path):
    for src in (MODULE, SNIPPET):
        pre = tmp_path / (os.path.basename(src)[:-4] + ".f90")
        with open(pre, "w") as out:
            subprocess.run(["cpp", "-traditional-cpp", "-P", src], stdout=out, check=True)
        r = subprocess.run([FLANG, "-c", str(pre), "-o", str(pre) + ".o"], cwd=tmp_path,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
