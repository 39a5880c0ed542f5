"""afivo .dat tree files (afivo/src/m_af_output.f90:41-374) and the
streamer's restart record (src/streamer.f90:117-138, 521-557).

* afh.datfile reads back what it writes, byte for byte;
* the reference's own af_read_tree + af_write_tree (oracle/_ref/dat_roundtrip,
  compiled from /root/reference; build container only) reproduces our file
  byte for byte -- the format is the reference's in both directions;
* a simulation written to a .dat file and restarted from it continues
  exactly as the uninterrupted run (C oracle here; the HIP library in the
  -m gpu twin, whose files equal the oracle's).
"""
import os
import subprocess

import numpy as np
import pytest

import golden
from afh import capi
from afh.datfile import DatTree, parse_sim_data
from afh.driver import Simulation

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUNDTRIP = os.path.join(REPO, "oracle", "_ref", "dat_roundtrip")


def _sim(lib, device=-1, steps=4):
    sim = Simulation(lib, golden.load("rtest_test_3d"), device=device)
    sim.start()
    for _ in range(steps):
        sim.step()
    return sim


@pytest.fixture(scope="module")
def oracle_run(tmp_path_factory):
    d = tmp_path_factory.mktemp("dat")
    sim = _sim(capi.oracle_library())
    sim.write_dat(str(d / "run"))
    return sim, d / "run.dat"


def test_read_write_identity(oracle_run):
    _, path = oracle_run
    raw = path.read_bytes()
    t = DatTree.read(path)
    assert t.to_bytes() == raw
    sd = parse_sim_data(t.other, 2)
    assert sd["it"] == 4 and sd["global_dt"] > 0


@pytest.mark.skipif(not os.path.exists(ROUNDTRIP), reason="needs oracle/_ref (build container)")
def test_reference_reads_and_writes_our_file(oracle_run, tmp_path):
    _, path = oracle_run
    out = tmp_path / "ref"
    subprocess.run([ROUNDTRIP, str(path), str(out), "1"], check=True,
                   stdout=subprocess.DEVNULL)
    assert (tmp_path / "ref.dat").read_bytes() == path.read_bytes()


@pytest.mark.skipif(not os.path.exists(ROUNDTRIP), reason="needs oracle/_ref (build container)")
def test_reference_roundtrip_without_other_data(oracle_run, tmp_path):
    _, path = oracle_run
    t = DatTree.read(path)
    t.other = None
    t.cc_write_binary[3] = False  # a variable left out of the file
    src = tmp_path / "plain.dat"
    t.write(src)
    subprocess.run([ROUNDTRIP, str(src), str(tmp_path / "ref"), "0"], check=True,
                   stdout=subprocess.DEVNULL)
    assert (tmp_path / "ref.dat").read_bytes() == src.read_bytes()


def _compare(a, b):
    assert a.af.highest_id == b.af.highest_id
    for bid in range(1, a.af.highest_id + 1):
        assert a.af.in_use[bid] == b.af.in_use[bid]
        if a.af.in_use[bid]:
            assert (a.af.lvl[bid], tuple(a.af.ix[bid]), a.af.parent[bid]) == \
                (b.af.lvl[bid], tuple(b.af.ix[bid]), b.af.parent[bid])
            assert list(a.af.children[bid]) == list(b.af.children[bid])
            assert list(a.af.neighbors[bid]) == list(b.af.neighbors[bid])
    for l in range(1, a.af.highest_lvl + 1):
        assert a.af.lvls[l] == b.af.lvls[l]
    used = [i - 1 for i in range(1, a.af.highest_id + 1) if a.af.in_use[i]]
    for iv in range(1, a.n_var_cell + 1):
        assert np.array_equal(a.tree.get_cc(iv)[used], b.tree.get_cc(iv)[used])
    for iv in range(1, a.n_var_face + 1):
        assert np.array_equal(a.tree.get_fc(iv)[used], b.tree.get_fc(iv)[used])
    for k in ("it", "output_cnt", "time", "global_time", "photoi_prev_time", "global_dt"):
        assert getattr(a, k) == getattr(b, k), k


def test_restart_continues_exactly(oracle_run):
    sim, path = oracle_run
    lib = capi.oracle_library()
    other = Simulation(lib, golden.load("rtest_test_3d"))
    other.restart(str(path))
    other.log = []
    _compare(sim, other)
    for _ in range(3):
        sim.step()
        other.step()
    _compare(sim, other)


@pytest.mark.gpu
def test_restart_hip(oracle_run, tmp_path):
    """The device tree written to and restarted from a .dat file: the HIP
    run's file has the oracle run's topology and its data to 1e-9 (the
    device and oracle runs agree to that, test_rtest), and a device restart
    from the oracle's file continues as the oracle does."""
    osim, opath = oracle_run
    sim = _sim(capi.hip_library(), device=0)
    sim.write_dat(str(tmp_path / "hip"))
    h, o = DatTree.read(tmp_path / "hip.dat"), DatTree.read(opath)
    assert h.lvls == o.lvls and sorted(h.boxes) == sorted(o.boxes)
    for bid, bo in o.boxes.items():
        bh = h.boxes[bid]
        assert (bh.ix, bh.parent, bh.children, bh.neighbors) == \
            (bo.ix, bo.parent, bo.children, bo.neighbors)
    for iv in range(1, o.n_var_cell + 1):
        a = np.stack([h.boxes[b].cc[iv] for b in sorted(o.boxes)])
        b = np.stack([o.boxes[b].cc[iv] for b in sorted(o.boxes)])
        assert np.max(np.abs(a - b)) <= 1e-9 * max(np.max(np.abs(b)), 1e-300), iv
    assert parse_sim_data(h.other, 2)["it"] == parse_sim_data(o.other, 2)["it"]
    dev = Simulation(capi.hip_library(), golden.load("rtest_test_3d"), device=0)
    dev.restart(str(opath))
    ref = Simulation(capi.oracle_library(), golden.load("rtest_test_3d"))
    ref.restart(str(opath))
    for _ in range(3):
        dev.step()
        ref.step()
    used = [i - 1 for i in range(1, ref.af.highest_id + 1) if ref.af.in_use[i]]
    for iv in ref.densities:
        a, b = dev.tree.get_cc(iv)[used], ref.tree.get_cc(iv)[used]
        rel = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
        assert rel <= 1e-9, (ref.cc_names[iv - 1], rel)
