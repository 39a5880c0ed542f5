"""Input decks of the bench and the driver configurations (package data,
arrays only): the transport / chemistry tables of the old-style air model
(tables_air_siglo.npz, scripts/make_decks.py) and the set-up of BASELINE
configs 1, 3, 4, 5 (case_s2d / case_s3 / case_s4 / case_s5.npz, exported by
oracle/_ref/export_case from the reference's own initializers,
oracle/make_cases.py)."""
import os

import numpy as np

DIR = os.path.dirname(os.path.abspath(__file__))


def path(name):
    return os.path.join(DIR, name + ".npz")


def has(name):
    return os.path.exists(path(name))


def load(name):
    return dict(np.load(path(name)))
