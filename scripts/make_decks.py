#!/usr/bin/env python3
"""The bench's physics inputs as package data (afivo-streamer_amd/afh/decks):
the transport and chemistry tables of the old-style air model
(td_air_siglo_swarm.txt as the reference's transport_data_initialize reads
it), taken from tests/golden/uni8.npz (oracle/_ref/golden_gen's export) --
arrays only. The driver configurations' decks (case_s3/s4/s5/s2d.npz,
exported by oracle/_ref/export_case from the reference's own initializers,
oracle/make_cases.py) live in the same directory.
"""
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("td_rows_cols", "td_xmin", "td_inv_fac", "chem_rows_cols", "chem_xmin", "chem_inv_fac")

g = np.load(os.path.join(REPO, "tests", "golden", "uni8.npz"))
np.savez_compressed(os.path.join(REPO, "afivo-streamer_amd", "afh", "decks",
                                 "tables_air_siglo.npz"), **{k: g[k] for k in KEYS})
