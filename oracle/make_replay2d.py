#!/usr/bin/env python3
"""ORACLE TEST INFRASTRUCTURE -- 2-D species-step fixtures (build container only).

For each 2-D state of tests/state2d.py (BASELINE config 1: streamer_2d.cfg
with air_chemistry_v1, and tests/test_2d.cfg's old-style model) this script
writes the state as a replay record, runs the reference's own forward_euler
on it (oracle/_ref/2d/replay_step: the NDIM = 2 build of the reference's
module set, flux_upwind_tree with the m_fluid callbacks, flux_update_densities
with add_source_terms / get_rates) for both Heun sub-steps, and packs the
reference's dt_lim and the interiors of every density of the output state on
the leaves into tests/golden/replay2d_<name>.npz. The state itself is not
stored: tests/test_2d_replay.py rebuilds it with the same code.

    make -C oracle _ref/2d/replay_step && python3 oracle/make_replay2d.py
"""
import os
import resource
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import state2d  # noqa: E402

EXE = os.path.join(HERE, "_ref", "2d", "replay_step")
CWD = {"s2d": ("/root/reference/programs/standard_2d", ["streamer_2d.cfg"]),
       "test_2d": ("/root/reference/programs/standard_2d/tests", ["test_2d.cfg"])}


def replay(name, stage, tmp):
    c, af, cc, fc, dt = state2d.build_state(name)
    rec, out = os.path.join(tmp, "rec.bin"), os.path.join(tmp, "out.bin")
    used = state2d.write_record(rec, af, cc, fc, dt, 0.0, stage)
    cwd, args = CWD[name]

    def unlimited_stack():
        resource.setrlimit(resource.RLIMIT_STACK,
                           (resource.RLIM_INFINITY, resource.RLIM_INFINITY))
    env = dict(os.environ, OMP_STACKSIZE="512M", OMP_NUM_THREADS="4")
    subprocess.run([EXE, rec, out] + args, cwd=cwd, check=True, stdout=subprocess.DEVNULL,
                   preexec_fn=unlimited_stack, env=env)
    raw = open(out, "rb").read()
    dt_lim = np.frombuffer(raw, np.float64, 1)[0]
    ng = af.nc + 2
    ref = np.frombuffer(raw, np.float64, offset=8).reshape(len(cc), len(used), ng, ng)
    leaves = set(af.leaves())
    li = [k for k, b in enumerate(used) if b in leaves]
    s_out = stage[3]
    dens = {}
    for iv in c.ia("all_densities"):
        dens[str(iv)] = ref[iv + s_out - 1][li][:, 1:-1, 1:-1].copy()
    return dt_lim, dens, [used[k] for k in li]


def main():
    if not os.path.exists(EXE):
        sys.exit("build %s first (make -C oracle _ref/2d/replay_step)" % EXE)
    names = sys.argv[1:] or sorted(state2d.SPECS)
    for name in names:
        out = {}
        with tempfile.TemporaryDirectory() as tmp:
            for k, stage in enumerate(state2d.STAGES):
                dt_lim, dens, leaves = replay(name, stage, tmp)
                out["stage%d_dt_lim" % k] = np.array([dt_lim])
                out["stage%d_leaves" % k] = np.array(leaves, np.int32)
                for iv, a in dens.items():
                    out["stage%d_iv%s" % (k, iv)] = a
        path = os.path.join(REPO, "tests", "golden", "replay2d_%s.npz" % name)
        np.savez_compressed(path, **out)
        print("wrote", path, {k: v.shape for k, v in out.items() if k.endswith("leaves")})


if __name__ == "__main__":
    main()
