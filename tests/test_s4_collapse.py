"""Config 4 to the end of its time loop: does the
reference's own streamer.f90 stop where afh.driver stops?

Fixtures (tests/golden/, made by scripts/s4_collapse_fixtures.sh):
- s4_collapse_ref_rtest.txt: the regression log of the reference's
  src/streamer.f90 itself, built from the reference sources and run through
  the shim on the C oracle (oracle/_ref/dropin_streamer, build container),
  on BASELINE config 4 (tests/test_dropin_streamer.py's S4 arguments,
  end_time = 2.5 ns, output%dt = 0.05 ns); s4_collapse_ref_stop.txt: the
  last lines it printed;
- s4_collapse_hip_rows.json: afh.driver's rows of the same run on the GPU
  (scripts/s4_timeloop_rows.py).

Both runs stop with "dt too small" (streamer.f90:357-378: the dielectric
relaxation limit falls below dt_min = 1e-14 s as n_e grows at the rod), and
both write a last regression row at that point. The CPU test compares the
committed rows; the GPU test reruns the device loop and compares it with the
reference's rows.
"""
import json
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
REF_LOG = os.path.join(GOLD, "s4_collapse_ref_rtest.txt")
REF_STOP = os.path.join(GOLD, "s4_collapse_ref_stop.txt")
HIP_ROWS = os.path.join(GOLD, "s4_collapse_hip_rows.json")
# measured 4.7e-8 over all 46 rows (the rows are printed in E20.8); the
# bound of the other regression-row tests
RTOL = 1e-7


def _ref():
    return np.loadtxt(REF_LOG, skiprows=1, ndmin=2)


def _compare(rows, ref):
    assert rows.shape == ref.shape, (rows.shape, ref.shape)
    rel = np.abs(rows - ref) / np.maximum(np.abs(ref), 1e-300)
    print("max rel per row", rel.max(axis=1))
    assert rel.max() <= RTOL, rel.max(axis=1)


def test_reference_program_stops_with_dt_too_small():
    text = open(REF_STOP).read()
    assert "dt too small" in text
    ref = _ref()
    # the last row is the one written at the stop, before the end time
    assert ref[-1, 1] < 2.5e-9


def test_device_rows_equal_reference_program_rows():
    dev = json.load(open(HIP_ROWS))
    assert dev["error"] == "dt too small"
    _compare(np.array(dev["rows"]), _ref())


@pytest.mark.gpu
def test_device_time_loop_to_the_collapse(tmp_path):
    import subprocess
    import sys
    out = tmp_path / "rows.json"
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "s4_timeloop_rows.py"),
                        str(out), "2.5e-9", "0.05e-9", "240"],
                       capture_output=True, text=True, timeout=290)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    dev = json.load(open(out))
    assert dev["error"] == "dt too small"
    _compare(np.array(dev["rows"]), _ref())
