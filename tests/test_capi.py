"""CPU-side checks of the C ABI: the product library builds for gfx950, loads,
and exports every symbol include/afivo_hip.h declares (no compute calls)."""
import ctypes

import pytest

from afh import capi


def test_header_declares_api():
    syms = capi.header_symbols()
    assert "afh_mg_fas_vcycle" in syms and "afh_flux_upwind_tree" in syms
    assert len(syms) >= 24


def test_hip_library_exports_every_header_symbol():
    lib = ctypes.CDLL(capi.HIP_LIB)
    missing = [s for s in capi.header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    bound = {"afh_" + n for n in capi.SIGNATURES}
    assert set(capi.header_symbols()) == bound


def test_oracle_exports_same_api():
    lib = ctypes.CDLL(capi.ORACLE_LIB)
    missing = [s.replace("afh_", "afo_") for s in capi.header_symbols()
               if not hasattr(lib, s.replace("afh_", "afo_"))]
    assert not missing, missing


def test_no_device_is_an_error_not_a_fallback():
    """Without a GPU the product must fail loudly (no CPU fallback)."""
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from afh.model import Tree
    from afh.tree import uniform_tree
    topo = uniform_tree(4, (4, 4, 4), (1e-3, 1e-3, 1e-3), 2)
    with pytest.raises(capi.AfhError):
        Tree(capi.hip_library(), topo, 14, 2)
