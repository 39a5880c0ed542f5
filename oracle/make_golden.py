#!/usr/bin/env python3
"""ORACLE TEST INFRASTRUCTURE -- pack golden vectors (build container only).

Runs the golden-vector harness (oracle/_ref/golden_gen, afivo numerics compiled
from /root/reference by oracle/Makefile) and packs its raw binary dumps into
tests/golden/<case>.npz. Usage:

    make -C oracle ref && python3 oracle/make_golden.py

Array conventions in the .npz (all float64 unless noted):
  meta_*      per-box topology, 1-based ids as in afivo (0 = no box, -1 = phys.)
  lvl_ids_<l>, lvl_leaves_<l>, lvl_parents_<l>   int32 id lists per level
  td_rows_cols (n_points, 4), td_xmin, td_inv_fac   transport table
  chem_rows_cols (n_points, 2), chem_xmin, chem_inv_fac
  <state>__<var>   cc array (n_boxes, nc+2, nc+2, nc+2) = [box][k][j][i]
  <state>__fc_<var> fc array (n_boxes, 3, nc+1, nc+1, nc+1) = [box][dim][k][j][i]
  trace states store only boxes that changed: <state>__<var>__ids (0-based)
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
TD_FILE = "/root/reference/transport_data/td_air_siglo_swarm.txt"

# cc variable indices (1-based, hx_physics.f90)
CC = {"e0": 1, "e1": 2, "e2": 3, "pos0": 4, "pos1": 5, "neg0": 7, "neg1": 8,
      "phi": 10, "efld": 12, "rhs": 13, "tmp": 14, "lsf": 15}
FC = {"flux": 1, "field": 2}

CHAIN = [
    ("init", ["e0", "pos0", "neg0", "phi"], []),
    ("rhs", ["rhs"], []),
    ("vcycle1", ["phi", "tmp", "rhs"], []),
    ("vcycle2", ["phi", "tmp", "rhs"], []),
    ("field0", ["efld"], ["field"]),
    ("flux1", ["e0"], ["flux"]),
    ("update1", ["e1", "pos1", "neg1"], []),
    ("field1", ["rhs", "phi", "tmp", "efld"], ["field"]),
    ("flux2", ["e1"], ["flux"]),
    ("update2", ["e0", "pos0", "neg0"], []),
]
# FAS-FMG, run by the harness after the chain from the state it dumps as
# fmg_in (so every case can replay it in isolation)
FMG = [
    ("fmg_in", ["e0", "pos0", "neg0", "phi", "rhs", "tmp"], []),
    ("fmg0", ["rhs", "phi", "tmp"], []),
    ("fmg1", ["rhs", "phi", "tmp"], []),
]
# Helmholtz FMG of a photoionization mode (lambda = 44081.25 1/m), run after
# FMG from the state dumped as helm_in
HELM = [
    ("helm_in", ["rhs", "phi", "tmp"], []),
    ("helm0", ["rhs", "phi", "tmp"], []),
    ("helm1", ["rhs", "phi", "tmp"], []),
]
HELM_LAMBDA = 44081.25
# rod electrode (level-set function): the field solve through the reference's
# LSF stencils, dumped in lsf.bin
ROD = [
    ("init", ["phi", "lsf"], []),
    ("rhs", ["rhs"], []),
    ("vcycle1", ["phi", "tmp", "rhs"], []),
    ("vcycle2", ["phi", "tmp", "rhs"], []),
    ("field0", ["efld"], ["field"]),
    ("fmg_in", ["phi", "rhs", "tmp"], []),
    ("fmg0", ["rhs", "phi", "tmp"], []),
    ("fmg1", ["rhs", "phi", "tmp"], []),
]
# one af_adjust_refinement (refine near a point, derefine far from it) on an
# AMR tree; "after_" keys hold the new topology (boxes not in use: lvl 0)
REGRID = [
    ("regrid_in", ["e0", "pos0", "neg0", "phi", "efld"], []),
]
REGRID_AFTER = ("regrid", ["e0", "pos0", "neg0", "phi", "efld"])
CASES = {
    "uni4": {"chain": CHAIN + FMG + HELM, "trace": True},
    "uni8": {"chain": CHAIN + FMG + HELM, "trace": False},
    "amr4": {"chain": CHAIN[:7] + FMG + HELM, "trace": False},
    "rod8": {"chain": ROD, "trace": False, "lsf": True},
    "regrid8": {"chain": REGRID, "trace": False, "regrid": True},
}


def read_topology(path, ndim=3):
    """ndim = 2: the 2-D harness' topology (golden_gen2d.f90): ix (n, 2),
    children (n, 4), neighbors (n, 4), neighbor_mat (n, 9), r_min / dr (n, 2)."""
    raw = open(path, "rb").read()
    off = 0

    def take(dtype, n):
        nonlocal off
        a = np.frombuffer(raw, dtype=dtype, count=n, offset=off)
        off += a.nbytes
        return a.copy()

    nc, nbox, nlvl, nvc, nvf = take(np.int32, 5)
    out = {"nc": nc, "n_boxes": nbox, "highest_lvl": nlvl, "n_var_cell": nvc,
           "n_var_face": nvf}
    d = ndim
    out["coarse_grid_size"] = take(np.int32, d)
    out["r_base"] = take(np.float64, d)
    out["dr_base"] = take(np.float64, d)
    lvl = np.zeros(nbox, np.int32)
    ix = np.zeros((nbox, d), np.int32)
    parent = np.zeros(nbox, np.int32)
    children = np.zeros((nbox, 2 ** d), np.int32)
    neighbors = np.zeros((nbox, 2 * d), np.int32)
    nmat = np.zeros((nbox, 3 ** d), np.int32)
    r_min = np.zeros((nbox, d))
    dr = np.zeros((nbox, d))
    for b in range(nbox):
        lvl[b] = take(np.int32, 1)[0]
        ix[b] = take(np.int32, d)
        parent[b] = take(np.int32, 1)[0]
        children[b] = take(np.int32, 2 ** d)
        neighbors[b] = take(np.int32, 2 * d)
        nmat[b] = take(np.int32, 3 ** d)
        r_min[b] = take(np.float64, d)
        dr[b] = take(np.float64, d)
    out.update(meta_lvl=lvl, meta_ix=ix, meta_parent=parent,
               meta_children=children, meta_neighbors=neighbors,
               meta_neighbor_mat=nmat, meta_r_min=r_min, meta_dr=dr)
    for lv in range(1, nlvl + 1):
        ni, nl, npar = take(np.int32, 3)
        out["lvl_ids_%d" % lv] = take(np.int32, ni)
        out["lvl_leaves_%d" % lv] = take(np.int32, nl)
        out["lvl_parents_%d" % lv] = take(np.int32, npar)
    cv, ngas = take(np.float64, 2)
    out["current_voltage"] = cv
    out["gas_number_density"] = ngas
    out["domain"] = take(np.float64, d)
    if d == 2:
        out["ndim"] = np.int32(2)
    return out


def read_tables(path):
    raw = open(path, "rb").read()
    off = 0
    out = {}
    for name in ("td", "chem"):
        npts, ncol = np.frombuffer(raw, np.int32, 2, off)
        off += 8
        xmin, inv = np.frombuffer(raw, np.float64, 2, off)
        off += 16
        rc = np.frombuffer(raw, np.float64, npts * ncol, off)
        off += rc.nbytes
        out[name + "_rows_cols"] = rc.reshape(ncol, npts).T.copy()
        out[name + "_xmin"] = xmin
        out[name + "_inv_fac"] = inv
    return out


def read_state(path, topo):
    nb, nc = int(topo["n_boxes"]), int(topo["nc"])
    nvc, nvf = int(topo["n_var_cell"]), int(topo["n_var_face"])
    d = int(topo.get("ndim", 3))
    a = np.fromfile(path, dtype=np.float64)
    ncc = nb * nvc * (nc + 2) ** d
    cc = a[:ncc].reshape((nb, nvc) + (nc + 2,) * d)
    fc = a[ncc:].reshape((nb, nvf, d) + (nc + 1,) * d)
    return cc, fc


def read_lsf(path, topo):
    """lsf.bin of golden_gen (dump_lsf): per box the variable operator
    stencil v(7, nc^3) + bc_correction, and the sparse boundary distances
    (sparse_ix(3, n), sparse_v(6, n)) with the boundary values.
      lsf_v_ids (m,) 1-based box ids; lsf_v (m, nc, nc, nc, 7) [k][j][i][c];
      lsf_bcc (m, nc, nc, nc) (zeros where lsf_bcc_has == 0)
      lsf_d_ids, lsf_d_n (q,); lsf_d_ix (sum n, 3) int32 (i, j, k, 1-based);
      lsf_d_dd (sum n, 6); lsf_d_bval (q, nc, nc, nc)"""
    nb, nc = int(topo["n_boxes"]), int(topo["nc"])
    raw = open(path, "rb").read()
    off = 0

    def take(dtype, n):
        nonlocal off
        a = np.frombuffer(raw, dtype=dtype, count=n, offset=off)
        off += a.nbytes
        return a.copy()

    n3 = nc ** 3
    v_ids, v, bcc, bcc_has = [], [], [], []
    d_ids, d_n, d_ix, d_dd, d_bv = [], [], [], [], []
    for b in range(nb):
        if take(np.int32, 1)[0]:
            v_ids.append(b + 1)
            v.append(take(np.float64, 7 * n3).reshape(nc, nc, nc, 7))
            has = take(np.int32, 1)[0]
            bcc_has.append(has)
            bcc.append(take(np.float64, n3).reshape(nc, nc, nc) if has
                       else np.zeros((nc, nc, nc)))
        n = take(np.int32, 1)[0]
        if n:
            d_ids.append(b + 1)
            d_n.append(n)
            d_ix.append(take(np.int32, 3 * n).reshape(n, 3))
            d_dd.append(take(np.float64, 6 * n).reshape(n, 6))
            d_bv.append(take(np.float64, n3).reshape(nc, nc, nc))
    assert off == len(raw)
    return {"lsf_v_ids": np.array(v_ids, np.int32), "lsf_v": np.array(v),
            "lsf_bcc": np.array(bcc), "lsf_bcc_has": np.array(bcc_has, np.int32),
            "lsf_d_ids": np.array(d_ids, np.int32), "lsf_d_n": np.array(d_n, np.int32),
            "lsf_d_ix": np.concatenate(d_ix).astype(np.int32),
            "lsf_d_dd": np.concatenate(d_dd), "lsf_d_bval": np.array(d_bv)}


# BASELINE config 1, the reference's 2-D build (oracle/_ref/2d/golden_gen2d):
# arrays are [box][j][i] (cc) and [box][dim][j][i] (fc)
CASES_2D = {
    "uni2d": {"chain": CHAIN + FMG + HELM, "trace": False, "ndim": 2},
    "amr2d": {"chain": CHAIN + FMG + HELM, "trace": False, "ndim": 2},
}


def pack(case, raw_dir):
    spec = CASES_2D[case] if case in CASES_2D else CASES[case]
    topo = read_topology(os.path.join(raw_dir, "topology.bin"), spec.get("ndim", 3))
    out = dict(topo)
    out.update(read_tables(os.path.join(raw_dir, "tables.bin")))
    # scalar logs (dt limits, residuals, thresholds)
    for line in open(os.path.join(raw_dir, "log.txt")):
        f = line.split()
        if not f or f[0] in ("state",):
            continue
        key = "log_" + f[0] + ("_%s" % f[1] if f[0] == "field1_residual" else "")
        vals = [float(x) for x in (f[2:] if f[0] == "field1_residual" else f[1:])]
        out[key] = np.array(vals)
    out["helm_lambda"] = np.array(HELM_LAMBDA)
    if spec.get("lsf"):
        out.update(read_lsf(os.path.join(raw_dir, "lsf.bin"), topo))
    if spec.get("regrid"):
        after = read_topology(os.path.join(raw_dir, "topology_after.bin"))
        in_use = np.fromfile(os.path.join(raw_dir, "in_use_after.bin"), np.int32)[1:]
        for k in ("meta_lvl", "meta_parent", "meta_children", "meta_neighbors",
                  "meta_neighbor_mat"):
            after[k][in_use == 0] = 0
        for k, v in after.items():
            out["after_" + k] = v
        raw = open(os.path.join(raw_dir, "refine.bin"), "rb").read()
        nbx = int(np.frombuffer(raw, np.int32, 1, 0)[0])
        out["refine_flags"] = np.frombuffer(raw, np.int32, nbx, 4).copy()
        out["refine_masks"] = np.frombuffer(raw, np.int32, nbx, 4 + 4 * nbx).copy()
        out["refine_params"] = np.frombuffer(raw, np.float64, 28, 4 + 8 * nbx).copy()
        out["refine_buffer"] = np.frombuffer(raw, np.int32, 1, 4 + 8 * nbx + 224).copy()
        name, ccv = REGRID_AFTER
        cc, _ = read_state(os.path.join(raw_dir, "state_%s.bin" % name), after)
        for v in ccv:
            out["%s__%s" % (name, v)] = cc[:, CC[v] - 1].copy()
    for name, ccv, fcv in spec["chain"]:
        cc, fc = read_state(os.path.join(raw_dir, "state_%s.bin" % name), topo)
        for v in ccv:
            out["%s__%s" % (name, v)] = cc[:, CC[v] - 1].copy()
        for v in fcv:
            out["%s__fc_%s" % (name, v)] = fc[:, FC[v] - 1].copy()
    if spec["trace"]:
        logged = [l.split()[1] for l in open(os.path.join(raw_dir, "log.txt"))
                  if l.split() and l.split()[0] == "state"]
        seq = ["rhs"] + [s for s in logged if s.startswith("tr_")]
        prev = read_state(os.path.join(raw_dir, "state_rhs.bin"), topo)[0]
        order = []
        for name in seq[1:]:
            cc = read_state(os.path.join(raw_dir, "state_%s.bin" % name), topo)[0]
            for v in ("phi", "rhs", "tmp"):
                i = CC[v] - 1
                changed = np.where(np.any(cc[:, i] != prev[:, i], axis=(1, 2, 3)))[0]
                out["%s__%s__ids" % (name, v)] = changed.astype(np.int32)
                out["%s__%s" % (name, v)] = cc[changed, i].copy()
            order.append(name)
            prev = cc
        out["trace_order"] = np.array(order)
    dst = os.path.join(REPO, "tests", "golden", case + ".npz")
    np.savez_compressed(dst, **out)
    return dst


def main():
    gen = os.path.join(HERE, "_ref", "golden_gen")
    if not os.path.exists(gen):
        sys.exit("build the harness first: make -C oracle ref")
    gen2d = os.path.join(HERE, "_ref", "2d", "golden_gen2d")
    for case in (sys.argv[1:] or list(CASES) + list(CASES_2D)):
        raw = os.path.join("/tmp", "golden_raw", case)
        os.makedirs(raw, exist_ok=True)
        for f in os.listdir(raw):
            os.remove(os.path.join(raw, f))
        subprocess.run([gen2d if case in CASES_2D else gen, case, TD_FILE, raw],
                       check=True, stdout=subprocess.DEVNULL)
        dst = pack(case, raw)
        print("%-5s -> %s (%.0f kB)" % (case, dst, os.path.getsize(dst) / 1e3))


if __name__ == "__main__":
    main()
