#!/usr/bin/env python3
"""The reference's own 2-D code timed on streamer_2d.cfg's set-up tree
(build container only): oracle/_ref/2d/ref_timing in
record mode reads the state scripts/record_setup_state.py wrote on the GPU
box from the device driver's set-up (the very tree bench.py --config 2d
runs), rebuilds that tree with the reference's af_adjust_refinement and
times forward_euler per Heun sub-step and one FAS V(2,2)-cycle without the
level-1 solve (HYPRE is absent), with OMP_NUM_THREADS = 1 and 8.

    python3 scripts/ref_cpu_timing_2d.py <record.bin> [tag]
Writes profiles/<tag>_ref_cpu_timing_2d.json.
"""
import json
import os
import resource
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROG = "/root/reference/programs/standard_2d"
EXE = os.path.join(REPO, "oracle", "_ref", "2d", "ref_timing")
sys.path.insert(0, os.path.join(REPO, "scripts"))
from ref_cpu_timing import cpu_model  # noqa: E402


def main(record, tag="r06", reps=20):
    def lim():
        resource.setrlimit(resource.RLIMIT_STACK, (resource.RLIM_INFINITY,) * 2)
    res = {"what": "the reference's own 2-D code (programs/standard_2d/streamer_2d.cfg, "
                   "air_chemistry_v1; oracle/_ref/2d/ref_timing, NDIM = 2, from "
                   "/root/reference) on streamer_2d.cfg's own set-up tree, read from a "
                   "record of the device driver's set-up (scripts/record_setup_state.py): "
                   "forward_euler per Heun sub-step and one FAS V(2,2)-cycle without the "
                   "level-1 solve",
           "command": "cd programs/standard_2d && OMP_NUM_THREADS=T "
                      "oracle/_ref/2d/ref_timing <record> %d streamer_2d.cfg" % reps,
           "cpu": cpu_model(),
           "measured_in": "the build container (the reference binary does not travel to "
                          "the GPU box)", "threads": {}}
    for th in (1, 8):
        env = dict(os.environ, OMP_NUM_THREADS=str(th), OMP_STACKSIZE="512M")
        out = subprocess.run([EXE, os.path.abspath(record), str(reps), "streamer_2d.cfg"],
                             cwd=PROG, env=env, capture_output=True, text=True, check=True,
                             preexec_fn=lim)
        f = [l for l in out.stdout.splitlines() if l.startswith("TIMING")][0].split()
        sp, vc, cells, boxes = float(f[2]), float(f[4]), int(f[6]), int(f[10])
        res["cells"], res["boxes"] = cells, boxes
        res["threads"][str(th)] = {"species_s": sp, "vcycle_s": vc, "unit_step_s": sp + vc,
                                   "cell_updates_per_s": cells / (sp + vc)}
        print(th, res["threads"][str(th)], flush=True)
    out = os.path.join(REPO, "profiles", "%s_ref_cpu_timing_2d.json" % tag)
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main(*sys.argv[1:])
