#!/usr/bin/env python3
"""ORACLE TEST INFRASTRUCTURE -- regression-case fixtures (build container only).

For each of the reference's 3D regression tests (programs/standard_3d/tests/
test_3d*.cfg, run by the reference's run_test.sh from that directory) this
script runs oracle/_ref/export_case (the reference's own module initializers,
compiled from /root/reference by oracle/Makefile) on the .cfg and packs what
it printed -- configuration values, variable registry, transport table,
parsed reactions, the field-rate lookup table, get_rates on a field grid --
together with the numbers of the reference's committed regression log for
that cfg (<name>_rtest.log: it, time, dt, volume-averaged sums and maxima of
every species per output time; the expected output) into
tests/golden/rtest_<name>.npz. Only numbers and names are stored.

    make -C oracle _ref/export_case && python3 oracle/make_cases.py [name ...]

The 2-D cases (BASELINE config 1: programs/standard_2d) use the NDIM = 2
build of the same harness (make -C oracle _ref/2d/export_case):
tests/golden/rtest_test_2d.npz (tests/test_2d.cfg with its regression log)
and afivo-streamer_amd/afh/decks/case_s2d.npz (streamer_2d.cfg itself:
air_chemistry_v1; the case_*.npz decks are package data the bench reads).
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
TESTS = "/root/reference/programs/standard_3d/tests"
CASES = ["test_3d", "test_3d_chem", "test_3d_photoi_chem"]
ION_ARGS = ["-input_data%mobile_ions=N2_plus O2_plus O2_min",
            "-input_data%ion_mobilities=1e-2 2e-2 1.5e-2"]
# BASELINE.json config 3: programs/standard_3d/streamer_3d.cfg with
# air_chemistry_v2 (9 species, 25 reactions); no regression log
EXTRA = {"s3": ("/root/reference/programs/standard_3d", "streamer_3d.cfg",
                ["-input_data%file=../../transport_data/air_chemistry_v2.txt",
                 "-input_data%old_style=f"]),
         # BASELINE.json config 4: config 3 with the rod electrode of
         # SURVEY.md 8(d) S4 (the geometry of the reference's own
         # standard_2d/tests/test_2d_pos_electrode.cfg: a grounded rod from
         # the z = 0 plane to 0.15 L, radius 1 mm), refined to 2e-4 m at
         # the electrode and to no less than 1e-4 m (5 levels of 8^3 boxes)
         "s4": ("/root/reference/programs/standard_3d", "streamer_3d.cfg",
                ["-input_data%file=../../transport_data/air_chemistry_v2.txt",
                 "-input_data%old_style=f", "-use_electrode=T",
                 "-field_electrode_grounded=T", "-field_rod_r0=0.5 0.5 0.0",
                 "-field_rod_r1=0.5 0.5 0.15", "-field_rod_radius=1e-3",
                 "-refine_electrode_dx=2e-4", "-refine_min_dx=1e-4"]),
         # BASELINE.json config 5: programs/3d_sprite/sprite_3d.cfg
         # (sprite_chemistry_v0, Helmholtz photoionization, the gas density
         # of its m_user.f90: an exponential atmosphere, so the "M" variable)
         "s5": ("/root/reference/programs/3d_sprite", "sprite_3d.cfg",
                ["--user-gas=sprite"]),
         # mobile ions (input_data%mobile_ions / ion_mobilities, flux species
         # 2.. of m_streamer.f90:253-282): test_3d_chem with three of its ions
         # made mobile, at the 1e-2 m^2/Vs of the reference's own
         # standard_2d/tests/test_cyl_ion_motion.cfg (far above real ion
         # mobilities, so the ion fluxes matter within a step)
         "ions": (TESTS, "test_3d_chem.cfg", ION_ARGS)}


TESTS_2D = "/root/reference/programs/standard_2d/tests"
CASES_2D = ["test_2d"]
EXTRA_2D = {"s2d": ("/root/reference/programs/standard_2d", "streamer_2d.cfg", [])}


def parse_dump(path):
    out = {}
    with open(path) as f:
        for line in f:
            kind, rest = line.split(":", 1)
            parts = rest.split()
            name, n = parts[0], int(parts[1])
            vals = parts[2:2 + n] if kind != "s" else None
            if kind == "r":
                out[name] = np.array([float(v.replace("D", "E")) for v in vals], np.float64)
            elif kind == "i":
                out[name] = np.array([int(v) for v in vals], np.int64)
            else:
                toks = rest.split(None, 2)[2] if n else ""
                if '"' in toks:
                    items = [t for t in toks.split('"') if t.strip()]
                else:
                    items = toks.split()
                out[name] = np.array(items[:n] if n else [], dtype="U64")
    return out


def main():
    only = set(sys.argv[1:])
    run(os.path.join(HERE, "_ref", "export_case"), TESTS, CASES, EXTRA, only)
    run(os.path.join(HERE, "_ref", "2d", "export_case"), TESTS_2D, CASES_2D, EXTRA_2D, only)


def run(exe, tests, cases, extra_cases, only):
    if only and not (only & (set(cases) | set(extra_cases))):
        return
    if not os.path.exists(exe):
        sys.exit("build %s first (make -C oracle %s)" % (exe, os.path.relpath(exe, HERE)))
    for name in cases:
        if only and name not in only:
            continue
        dump = "/tmp/afh_export_%s.txt" % name
        subprocess.run([exe, dump, name + ".cfg"], cwd=tests, check=True,
                       stdout=subprocess.DEVNULL)
        d = parse_dump(dump)
        log = os.path.join(tests, name + "_rtest.log")
        with open(log) as f:
            header = f.readline().split()
        d["rtest_columns"] = np.array(header, dtype="U64")
        d["rtest_log"] = np.genfromtxt(log, skip_header=1)
        out = os.path.join(REPO, "tests", "golden", "rtest_%s.npz" % name)
        np.savez_compressed(out, **d)
        os.remove(dump)
        print("wrote", out, len(d), "arrays")
    for name, (cwd, cfg, extra) in extra_cases.items():
        if only and name not in only:
            continue
        dump = "/tmp/afh_export_%s.txt" % name
        subprocess.run([exe, dump, cfg] + extra, cwd=cwd, check=True,
                       stdout=subprocess.DEVNULL)
        d = parse_dump(dump)
        # (input decks of the bench: package data)
        out = os.path.join(REPO, "afivo-streamer_amd", "afh", "decks", "case_%s.npz" % name)
        np.savez_compressed(out, **d)
        os.remove(dump)
        print("wrote", out, len(d), "arrays")


if __name__ == "__main__":
    main()
