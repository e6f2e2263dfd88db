"""CPU checks of the C-ABI library: it loads and exports every symbol that
include/dpf_hip.h declares (no compute calls without a GPU)."""
import ctypes

from distributed_point_functions_amd import hip_abi


def test_header_declares_hot_path_entry_points():
    fns = hip_abi.header_functions()
    for f in ("dpf_hip_hash", "dpf_hip_eval_paths", "dpf_hip_expand", "dpf_hip_eval_points"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = hip_abi.load()
    missing = [f for f in hip_abi.header_functions() if not hasattr(lib, f)]
    assert missing == []


def test_abi_version_and_packed_size():
    lib = hip_abi.load()
    assert lib.dpf_hip_abi_version() == 1
    d = hip_abi.value_desc([(hip_abi.LEAF_INT, 32, 0), (hip_abi.LEAF_INT, 64, 0)], True, 1, 1)
    assert lib.dpf_hip_packed_element_size(ctypes.byref(d)) == 12


def test_argument_validation_without_gpu():
    # Validation happens before any device work, so it is testable on CPU.
    lib = hip_abi.load()
    d = hip_abi.value_desc([(hip_abi.LEAF_INT, 4, 0)], True, 32, 1)
    k = hip_abi.aes_key(0)
    st = lib.dpf_hip_expand(1, None, None, 3, None, None, None, ctypes.byref(k), ctypes.byref(k),
                            ctypes.byref(k), ctypes.byref(d), 1, None, 0, None, None)
    assert st == 12  # UNIMPLEMENTED: 4-bit leaves have no C++ type in the reference
    assert b"power of two" in lib.dpf_hip_last_error()
    st = lib.dpf_hip_hash(-1, None, ctypes.byref(k), None, None)
    assert st == 3
