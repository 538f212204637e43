"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/koordgpu.h declares, and its
struct layouts match the binding.  No compute calls (no GPU here)."""
import ctypes
import os
import re

import numpy as np

from koordinator_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "koordgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(kg_[a-z_0-9]+)\s*\(", src))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(abi.LIB_PATH)
    declared = _header_functions()
    assert declared == set(abi.EXPORTED_SYMBOLS), declared ^ set(abi.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name


def test_struct_layouts_and_version():
    lib = abi.load_library()
    assert lib.kg_abi_version() == abi.ABI_VERSION
    for which, dt in abi.STRUCT_DTYPES.items():
        assert lib.kg_abi_struct_size(which) == dt.itemsize


def test_config_default_matches_v1beta2_defaults():
    from koordinator_amd import engine, framework
    c = engine.default_config()[0]
    # pkg/scheduler/apis/config/v1beta2/defaults.go:30-48,76-99
    assert c["la_filter_expired_node_metrics"] == 1
    assert c["la_node_metric_expiration_seconds"] == 180
    assert list(c["la_resource_weights"][:2]) == [1, 1]
    assert list(c["la_usage_thresholds"][:2]) == [65, 95]
    assert list(c["la_estimated_scaling_factors"][:2]) == [85, 70]
    assert c["la_score_according_prod_usage"] == 0
    f = framework.build_config()[0]
    for k in ("la_resource_weights", "la_usage_thresholds", "la_estimated_scaling_factors", "fit_resource_weights"):
        assert np.array_equal(c[k], f[k]), k


def test_missing_library_fails_loudly(tmp_path):
    import pytest
    with pytest.raises(RuntimeError, match="not built"):
        abi.load_library(str(tmp_path / "nope.so"))


def test_invalid_config_rejected_without_device():
    """kg_engine_create validates the config before touching the device."""
    from koordinator_amd import framework
    lib = abi.load_library()
    cfg = framework.build_config()
    cfg[0]["abi_version"] = 99
    h = ctypes.c_void_p()
    rc = lib.kg_engine_create(abi.ptr(cfg), 100, 0, 1, None, ctypes.byref(h))
    assert rc == abi.E_INVALID and b"abi_version" in lib.kg_last_error()
    cfg = framework.build_config()
    cfg[0]["fit_resource_weights"][abi.RES_EPHEMERAL] = 1
    assert lib.kg_engine_create(abi.ptr(cfg), 100, 0, 1, None, ctypes.byref(h)) == abi.E_UNSUPPORTED
