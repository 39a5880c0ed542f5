"""Drop-in check through the Fortran ISO_C_BINDING shim.

tests/fortran/dropin_heun.F90 is an afivo driver built from the reference
sources (oracle/Makefile `dropin`, build container only; the binaries travel
in oracle/_ref/). It sets up trees with the reference afivo API, runs every
stage of one Heun step with the reference routines and through the shim, and
requires bitwise-equal results:

* CPU: the shim bound to the C oracle (symbol prefix afo_);
* GPU: the shim bound to libafivo_hip.so (symbol prefix afh_).

The transport/chemistry tables come from the golden fixture (written here in
the layout of golden_gen's dump_tables).
"""
import os
import subprocess

import numpy as np
import pytest

import golden

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref")


def _tables(tmp_path):
    g = golden.load("uni8")
    path = tmp_path / "tables.bin"
    with open(path, "wb") as f:
        for name in ("td", "chem"):
            rc = np.asarray(g[name + "_rows_cols"], dtype=np.float64)
            np.array(rc.shape, dtype=np.int32).tofile(f)
            np.array([g[name + "_xmin"], g[name + "_inv_fac"]], np.float64).tofile(f)
            np.asfortranarray(rc).T.reshape(-1).tofile(f)  # column-major
    return str(path)


def _run(variant, case, tmp_path):
    exe = os.path.join(REF, variant, "dropin_heun")
    if not os.path.exists(exe):
        pytest.skip("drop-in driver not built (oracle/Makefile dropin needs "
                    "the reference sources)")
    dump = str(tmp_path / ("mg_%s.bin" % variant))
    out = subprocess.run([exe, case, _tables(tmp_path), dump], capture_output=True,
                         text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert out.returncode == 0 and "DROPIN OK" in out.stdout, out.stdout + out.stderr
    return out.stdout, np.fromfile(dump, np.float64)


@pytest.mark.parametrize("case", ["uni8", "amr4"])
def test_dropin_oracle(case, tmp_path):
    _, mg = _run("afo", case, tmp_path)
    assert mg.size and np.all(np.isfinite(mg))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uni8", "amr4"])
def test_dropin_hip(case, tmp_path):
    """The device-bound build: every stage bitwise against the reference
    routines, and FMG + V-cycle through the shim bitwise equal to the
    oracle-bound build's (the oracle build runs on the host CPU)."""
    _, mg = _run("afh", case, tmp_path)
    _, ref = _run("afo", case, tmp_path)
    assert np.array_equal(mg, ref)
