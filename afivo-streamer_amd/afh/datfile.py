"""afivo's binary tree files (.dat) -- af_write_tree / af_read_tree
(afivo/src/m_af_output.f90:41-374, af_dat_file_version = 3, NDIM = 3) and the
streamer's simulation record appended to them (write_sim_data /
read_sim_data, src/streamer.f90:521-557, datfile_version = 30).

The file is a Fortran stream (no record markers) in the compiler's native
layout: default integers and logicals are 4 bytes (gfortran: .true. = 1),
reals are float64, character names af_nlen = 20 bytes, little endian. Every
field the reference writes is kept, including the parts this library does
not use (stored boundary values, multigrid stencils, user tags), so a file
read here and written again is byte-identical (tests/test_datfile.py checks
that the reference's own af_read_tree + af_write_tree reproduces our files
byte for byte).

``DatTree`` is the in-memory image; ``DatTree.aftree()`` gives the host
topology (afh.amr.AfTree) from which a device tree is created, and
``afh.driver.Simulation.write_dat`` / ``restart`` move the cell and face data
between a file and the device.
"""
import numpy as np

from .amr import AfTree, MAX_LVL

AF_DAT_FILE_VERSION = 3
DATFILE_VERSION = 30        # src/streamer.f90:28
AF_NLEN = 20                # m_af_types.f90:72
AF_MAX_NUM_VARS = 1024      # m_af_types.f90:20
AF_XYZ = 0                  # coordinate type (m_af_types.f90)


class _Reader:
    def __init__(self, raw):
        self.raw, self.p = raw, 0

    def take(self, dtype, n=1):
        a = np.frombuffer(self.raw, dtype, n, self.p)
        self.p += a.nbytes
        return a

    def i(self, n=None):
        a = self.take("<i4", 1 if n is None else n)
        return int(a[0]) if n is None else a.astype(np.int64)

    def l(self, n=None):
        a = self.take("<i4", 1 if n is None else n)
        return bool(a[0]) if n is None else a != 0

    def d(self, n=None):
        a = self.take("<f8", 1 if n is None else n)
        return float(a[0]) if n is None else a.copy()

    def s(self, n, length=AF_NLEN):
        b = self.take("S%d" % length, n)
        return [x.decode("latin-1") for x in b]


class _Writer:
    def __init__(self):
        self.parts = []

    def i(self, v):
        self.parts.append(np.asarray(v, "<i4").tobytes())

    def l(self, v):
        self.parts.append(np.asarray(v, bool).astype("<i4").tobytes())

    def d(self, v):
        self.parts.append(np.asarray(v, "<f8").tobytes())

    def s(self, names, length=AF_NLEN):
        self.parts.append(b"".join(n.encode("latin-1")[:length].ljust(length)
                                   for n in names))

    def raw(self, b):
        self.parts.append(b)

    def bytes(self):
        return b"".join(self.parts)


class DatBox:
    """One box record (box_t fields as af_write_tree writes them)."""

    __slots__ = ("n_cell", "lvl", "tag", "ix", "parent", "children", "neighbors",
                 "neighbor_mat", "dr", "r_min", "coord_t", "cc", "fc", "bc", "stencils")


class DatTree:
    """af_t as stored in a .dat file (m_af_types.f90:326-393)."""

    def __init__(self):
        self.ready = True
        self.box_limit = 0
        self.highest_lvl = self.highest_id = 0
        self.n_cell = self.n_var_cell = self.n_var_face = 0
        self.coord_t = AF_XYZ
        self.coarse_grid_size = [0, 0, 0]
        self.periodic = [False] * 3
        self.r_base = np.zeros(3)
        self.dr_base = np.zeros(3)
        self.cc_names = [""] * AF_MAX_NUM_VARS
        self.fc_names = [""] * AF_MAX_NUM_VARS
        self.cc_num_copies = np.ones(AF_MAX_NUM_VARS, np.int64)
        self.cc_write_output = np.ones(AF_MAX_NUM_VARS, bool)
        self.cc_write_binary = np.ones(AF_MAX_NUM_VARS, bool)
        self.fc_write_binary = np.ones(AF_MAX_NUM_VARS, bool)
        self.removed_ids = []
        self.lvls = []          # per level 1..highest_lvl: (ids, leaves, parents)
        self.boxes = {}         # id -> DatBox (boxes in use)
        self.other = None       # bytes after the tree (write_other_data), or None

    # ------------------------------------------------------------------ I/O
    @classmethod
    def read(cls, path):
        """af_read_tree (m_af_output.f90:197-374)."""
        with open(path, "rb") as f:
            r = _Reader(f.read())
        t = cls()
        version = r.i()
        if version != AF_DAT_FILE_VERSION:
            raise ValueError("af_read_tree: incompatible file versions (%d, need %d)"
                             % (version, AF_DAT_FILE_VERSION))
        t.ready = r.l()
        t.box_limit, t.highest_lvl, t.highest_id = r.i(), r.i(), r.i()
        t.n_cell, t.n_var_cell, t.n_var_face, t.coord_t = r.i(), r.i(), r.i(), r.i()
        t.coarse_grid_size = [int(x) for x in r.i(3)]
        t.periodic = [bool(x) for x in r.l(3)]
        t.r_base, t.dr_base = r.d(3), r.d(3)
        t.cc_names, t.fc_names = r.s(AF_MAX_NUM_VARS), r.s(AF_MAX_NUM_VARS)
        t.cc_num_copies = r.i(AF_MAX_NUM_VARS)
        t.cc_write_output = r.l(AF_MAX_NUM_VARS)
        t.cc_write_binary = r.l(AF_MAX_NUM_VARS)
        t.fc_write_binary = r.l(AF_MAX_NUM_VARS)
        n = r.i()
        t.removed_ids = [int(x) for x in r.i(n)]
        for _ in range(t.highest_lvl):
            lv = []
            for _ in range(3):
                n = r.i()
                lv.append([int(x) for x in r.i(n)])
            t.lvls.append(tuple(lv))
        nc = t.n_cell
        ng, nf = nc + 2, nc + 1
        ncc = [n for n in range(t.n_var_cell) if t.cc_write_binary[n]]
        nfc = [n for n in range(t.n_var_face) if t.fc_write_binary[n]]
        for bid in range(1, t.highest_id + 1):
            if not r.l():
                continue
            b = DatBox()
            b.n_cell, n_bc, n_st = r.i(), r.i(), r.i()
            b.lvl, b.tag = r.i(), r.i()
            b.ix = tuple(int(x) for x in r.i(3))
            b.parent = r.i()
            b.children = [int(x) for x in r.i(8)]
            b.neighbors = [int(x) for x in r.i(6)]
            b.neighbor_mat = [int(x) for x in r.i(27)]
            b.dr, b.r_min = r.d(3), r.d(3)
            b.coord_t = r.i()
            b.cc = {n + 1: r.d(ng ** 3).reshape(ng, ng, ng) for n in ncc}
            b.fc = {n + 1: r.d(3 * nf ** 3).reshape(3, nf, nf, nf) for n in nfc}
            b.bc = None
            if n_bc > 0:
                nv = t.n_var_cell
                b.bc = {"index_to_nb": r.i(n_bc), "nb_to_index": r.i(6),
                        "type": r.i(nv * n_bc), "val": r.d(nc * nc * nv * n_bc),
                        "coords": r.d(3 * nc * nc * n_bc)}
            b.stencils = [_read_stencil(r, nc) for _ in range(n_st)]
            t.boxes[bid] = b
        present = r.l()
        t.other = r.raw[r.p:] if present else None
        return t

    def to_bytes(self):
        """af_write_tree (m_af_output.f90:41-194) + the other data."""
        w = _Writer()
        w.i(AF_DAT_FILE_VERSION)
        w.l(self.ready)
        w.i([self.box_limit, self.highest_lvl, self.highest_id, self.n_cell,
             self.n_var_cell, self.n_var_face, self.coord_t])
        w.i(self.coarse_grid_size)
        w.l(self.periodic)
        w.d(self.r_base)
        w.d(self.dr_base)
        w.s(self.cc_names)
        w.s(self.fc_names)
        w.i(self.cc_num_copies)
        w.l(self.cc_write_output)
        w.l(self.cc_write_binary)
        w.l(self.fc_write_binary)
        w.i(len(self.removed_ids))
        w.i(self.removed_ids)
        for lv in self.lvls:
            for ids in lv:
                w.i(len(ids))
                w.i(ids)
        ncc = [n + 1 for n in range(self.n_var_cell) if self.cc_write_binary[n]]
        nfc = [n + 1 for n in range(self.n_var_face) if self.fc_write_binary[n]]
        for bid in range(1, self.highest_id + 1):
            b = self.boxes.get(bid)
            w.l(b is not None)
            if b is None:
                continue
            n_bc = len(b.bc["index_to_nb"]) if b.bc is not None else 0
            w.i([b.n_cell, n_bc, len(b.stencils), b.lvl, b.tag])
            w.i(b.ix)
            w.i(b.parent)
            w.i(b.children)
            w.i(b.neighbors)
            w.i(b.neighbor_mat)
            w.d(b.dr)
            w.d(b.r_min)
            w.i(b.coord_t)
            for n in ncc:
                w.d(b.cc[n])
            for n in nfc:
                w.d(b.fc[n])
            if n_bc:
                w.i(b.bc["index_to_nb"])
                w.i(b.bc["nb_to_index"])
                w.i(b.bc["type"])
                w.d(b.bc["val"])
                w.d(b.bc["coords"])
            for st in b.stencils:
                w.raw(st)
        w.l(self.other is not None)
        if self.other is not None:
            w.raw(self.other)
        return w.bytes()

    def write(self, path):
        with open(path, "wb") as f:
            f.write(self.to_bytes())

    # ------------------------------------------------------------ topology
    def aftree(self):
        """The host topology (afh.amr.AfTree) of this tree, box ids as stored."""
        if self.coord_t != AF_XYZ:
            raise NotImplementedError("only Cartesian (af_xyz) trees")
        nc = self.n_cell
        dom = self.r_base + self.dr_base * np.asarray(self.coarse_grid_size, float)
        af = AfTree(nc, dom, self.coarse_grid_size, periodic=self.periodic,
                    r_min=self.r_base, box_limit=max(self.box_limit, self.highest_id))
        af.dr_base = np.asarray(self.dr_base, float).copy()
        af._grow(self.highest_id)
        for bid in range(1, len(af.in_use)):
            af.in_use[bid] = False
        for bid, b in self.boxes.items():
            af.in_use[bid] = True
            af.lvl[bid] = b.lvl
            af.ix[bid] = tuple(b.ix)
            af.parent[bid] = b.parent
            af.children[bid] = list(b.children)
            af.neighbors[bid] = list(b.neighbors)
            af.nmat[bid] = list(b.neighbor_mat)
            af.r_min[bid] = np.asarray(b.r_min, float).copy()
            af.dr[bid] = np.asarray(b.dr, float).copy()
        af.highest_id = self.highest_id
        af.highest_lvl = self.highest_lvl
        af.removed_ids = list(self.removed_ids)
        af.lvls = [None] + [{"ids": [], "leaves": [], "parents": []} for _ in range(MAX_LVL)]
        for lvl, (ids, leaves, parents) in enumerate(self.lvls, start=1):
            af.lvls[lvl] = {"ids": list(ids), "leaves": list(leaves), "parents": list(parents)}
        return af

    @classmethod
    def from_aftree(cls, af, cc_names, fc_names, cc_num_copies=None, box_limit=None):
        """A tree image of topology `af` (boxes as af_init_box leaves them:
        data zero, stored boundary values zero, face coordinates set, no
        stencils); fill ``boxes[id].cc`` / ``.fc`` before writing."""
        t = cls()
        nc = af.nc
        t.box_limit = int(box_limit if box_limit is not None else af.box_limit)
        t.highest_lvl, t.highest_id = af.highest_lvl, af.highest_id
        t.n_cell, t.n_var_cell, t.n_var_face = nc, len(cc_names), len(fc_names)
        t.coarse_grid_size = list(af.coarse_grid_size)
        t.periodic = list(af.periodic)
        t.r_base, t.dr_base = np.asarray(af.r_base, float), np.asarray(af.dr_base, float)
        t.cc_names = list(cc_names) + [""] * (AF_MAX_NUM_VARS - len(cc_names))
        t.fc_names = list(fc_names) + [""] * (AF_MAX_NUM_VARS - len(fc_names))
        if cc_num_copies is not None:
            t.cc_num_copies[:len(cc_num_copies)] = cc_num_copies
        t.removed_ids = list(af.removed_ids)
        t.lvls = [(list(af.lvls[l]["ids"]), list(af.lvls[l]["leaves"]),
                   list(af.lvls[l]["parents"])) for l in range(1, af.highest_lvl + 1)]
        ng, nf = nc + 2, nc + 1
        for bid in range(1, af.highest_id + 1):
            if not af.in_use[bid]:
                continue
            b = DatBox()
            b.n_cell, b.lvl, b.tag = nc, af.lvl[bid], AF_INIT_TAG
            b.ix = tuple(af.ix[bid])
            b.parent = af.parent[bid]
            b.children = list(af.children[bid])
            b.neighbors = list(af.neighbors[bid])
            b.neighbor_mat = list(af.nmat[bid])
            b.dr = np.asarray(af.dr[bid], float)
            b.r_min = np.asarray(af.r_min[bid], float)
            b.coord_t = AF_XYZ
            b.cc = {n: np.zeros((ng, ng, ng)) for n in range(1, t.n_var_cell + 1)}
            b.fc = {n: np.zeros((3, nf, nf, nf)) for n in range(1, t.n_var_face + 1)}
            b.bc = _init_bc(b, t.n_var_cell)
            b.stencils = []
            t.boxes[bid] = b
        return t


AF_INIT_TAG = -(2 ** 31) + 1  # af_init_tag = -huge(1) (m_af_types.f90)


def _init_bc(b, n_var_cell):
    """Boundary storage as af_init_box (m_af_core.f90:539-580) leaves it: one
    entry per physical face (neighbour < af_no_box = 0), type and value zero,
    face coordinates from af_get_face_coords (m_af_types.f90:1215-1253)."""
    faces = [nb for nb in range(1, 7) if b.neighbors[nb - 1] < 0]
    if not faces:
        return None
    nc = b.n_cell
    nb_to = np.zeros(6, np.int64)
    coords = np.zeros((len(faces), nc * nc, 3))
    for q, nb in enumerate(faces, start=1):
        nb_to[nb - 1] = q
        d = (nb - 1) // 2
        low = (nb - 1) % 2 == 0
        bc_dim = [x for x in range(3) if x != d]
        rmin = np.zeros(3)
        for x in bc_dim:
            rmin[x] = b.r_min[x] + 0.5 * b.dr[x]
        rmin[d] = b.r_min[d] if low else b.r_min[d] + nc * b.dr[d]
        ix = 0
        for j in range(1, nc + 1):
            for i in range(1, nc + 1):
                coords[q - 1, ix, bc_dim[0]] = rmin[bc_dim[0]] + (i - 1) * b.dr[bc_dim[0]]
                coords[q - 1, ix, bc_dim[1]] = rmin[bc_dim[1]] + (j - 1) * b.dr[bc_dim[1]]
                coords[q - 1, ix, d] = rmin[d]
                ix += 1
    return {"index_to_nb": np.array(faces, np.int64), "nb_to_index": nb_to,
            "type": np.zeros(n_var_cell * len(faces), np.int64),
            "val": np.zeros(nc * nc * n_var_cell * len(faces)),
            "coords": coords.reshape(-1)}


def _read_stencil(r, nc):
    """One stencil_t record (m_af_output.f90:129-177), kept as raw bytes."""
    p0 = r.p
    r.i(3)          # key, shape, stype
    r.l()           # cylindrical_gradient
    k = r.i()
    if k > 0:
        r.d(k)      # c
    k = r.i()
    if k > 0:
        r.d(k * nc ** 3)    # v(k, nc, nc, nc)
    if r.i() > 0:
        r.d(nc ** 3)        # f
    if r.i() > 0:
        r.d(nc ** 3)        # bc_correction
    k = r.i()
    if k > 0:
        r.i(3 * k)          # sparse_ix(NDIM, k)
    m = r.i()
    if k > 0 and m > 0:
        r.d(m * k)          # sparse_v(m, k)
    return r.raw[p0:r.p]


# ---------------------------------------------------------------- streamer
def sim_data_bytes(it, output_cnt, time, global_time, photoi_prev_time, global_dt,
                   global_rates, global_JdotE, fraction_steps_rejected):
    """write_sim_data (src/streamer.f90:521-536)."""
    w = _Writer()
    w.i([DATFILE_VERSION, it, output_cnt])
    w.d([time, global_time, photoi_prev_time, global_dt])
    w.d(np.asarray(global_rates, float))
    w.d([global_JdotE, fraction_steps_rejected])
    return w.bytes()


def parse_sim_data(raw, n_reactions):
    """read_sim_data (src/streamer.f90:538-557)."""
    r = _Reader(raw)
    if r.i() != DATFILE_VERSION:
        raise ValueError("Different datfile version")
    d = {"it": r.i(), "output_cnt": r.i(), "time": r.d(), "global_time": r.d(),
         "photoi_prev_time": r.d(), "global_dt": r.d(),
         "global_rates": r.d(n_reactions), "global_JdotE": r.d(),
         "fraction_steps_rejected": r.d()}
    if r.p != len(raw):
        raise ValueError("sim data: %d trailing bytes" % (len(raw) - r.p))
    return d
