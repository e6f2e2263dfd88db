"""ctypes binding of the C ABI in ``include/dpf_hip.h`` (``lib/libdpf_hip.so``).

Device buffers are torch tensors (torch is plumbing here: device memory,
streams, ``torch.distributed``); every compute call goes to the hand-written
gfx950 kernels.  There is no CPU fallback: if the shared library is missing
or no GPU is visible, calls raise.

torch is imported *before* the library is loaded so that both share one HIP
runtime (torch ships ``libamdhip64.so.7`` with the same SONAME).
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPF_HIP_LIB") or os.path.join(_HERE, "lib", "libdpf_hip.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "dpf_hip.h")
MAX_LEAVES = 16
LEAF_INT, LEAF_INTMODN, LEAF_XOR = 0, 1, 2
MASK64 = (1 << 64) - 1

_lib = None


class DpfHipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class Block(ctypes.Structure):
    _fields_ = [("low", ctypes.c_uint64), ("high", ctypes.c_uint64)]


class AesKey(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_uint8 * 16)]


class ValueDesc(ctypes.Structure):
    _fields_ = [
        ("num_leaves", ctypes.c_int32),
        ("direct", ctypes.c_int32),
        ("elements_per_block", ctypes.c_int32),
        ("blocks_needed", ctypes.c_int32),
        ("kind", ctypes.c_int32 * MAX_LEAVES),
        ("bits", ctypes.c_int32 * MAX_LEAVES),
        ("mod_low", ctypes.c_uint64 * MAX_LEAVES),
        ("mod_high", ctypes.c_uint64 * MAX_LEAVES),
    ]


def header_functions() -> list:
    """Names of every function the C ABI header declares."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(dpf_hip_\w+)\s*\(", txt, re.M)))


def load(require_gpu: bool = False):
    """Loads libdpf_hip.so (after torch, to share its HIP runtime)."""
    global _lib
    if _lib is None:
        try:
            import torch  # noqa: F401  (shared HIP runtime)
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise DpfHipError(13, f"HIP extension not built: {LIB_PATH} "
                                  "(run python -m distributed_point_functions_amd.build_native)")
        L = ctypes.CDLL(LIB_PATH)
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.dpf_hip_last_error.restype = ctypes.c_char_p
        L.dpf_hip_last_expand_kernel.restype = ctypes.c_char_p
        L.dpf_hip_last_expand_kernel.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.dpf_hip_last_batch_kernel.restype = ctypes.c_char_p
        L.dpf_hip_last_batch_kernel.argtypes = []
        L.dpf_hip_last_points_kernel.restype = ctypes.c_char_p
        L.dpf_hip_last_points_kernel.argtypes = []
        L.dpf_hip_hash.argtypes = [I64, P, P, P, P]
        L.dpf_hip_eval_paths.argtypes = [I64, I, P, P, P, P, P, P, P, P, P, P, P]
        L.dpf_hip_expand.argtypes = [I64, P, P, I, P, P, P, P, P, P, P, I, P, I, P, P]
        L.dpf_hip_eval_points.argtypes = [I64, I64, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P,
                                          P, P]
        L.dpf_hip_gather.argtypes = [I64, I64, I, P, P, P, P]
        L.dpf_hip_sum_shares_u64.argtypes = [I64, I64, I, I, P, P, P]
        L.dpf_hip_packed_element_size.argtypes = [P]
        L.dpf_hip_event_create.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        L.dpf_hip_event_destroy.argtypes = [P]
        L.dpf_hip_event_record.argtypes = [P, P]
        L.dpf_hip_event_elapsed_ms.argtypes = [P, P, ctypes.POINTER(ctypes.c_float)]
        L.dpf_hip_stream_sync.argtypes = [P]
        L.dpf_hip_clock_probe.argtypes = [I]
        L.dpf_hip_clock_probe_read.argtypes = [ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(ctypes.c_int64),
                                               ctypes.POINTER(ctypes.c_double)]
        _lib = L
    if require_gpu:
        import torch
        if not torch.cuda.is_available():
            raise DpfHipError(13, "no GPU visible: the DPF engine has no CPU fallback")
    return _lib


def last_expand_kernel():
    """(kernel, subtree depth) of this thread's last dpf_hip_expand launch,
    e.g. ("octet/mod32", 3) -- dispatch diagnostics for the tests."""
    d = ctypes.c_int(-1)
    name = load().dpf_hip_last_expand_kernel(ctypes.byref(d)).decode()
    return name, d.value


def last_batch_kernel() -> str:
    """Kernel of this thread's last batched prefix evaluation, e.g. "hh_level"
    -- dispatch diagnostics for the tests."""
    return load().dpf_hip_last_batch_kernel().decode()


def last_points_kernel() -> str:
    """Kernel of this thread's last point evaluation, e.g. "points/ilp4" --
    dispatch diagnostics for the tests."""
    return load().dpf_hip_last_points_kernel().decode()


def clock_probe(on: bool) -> None:
    """Turns the expand launches' in-kernel clock probe on (zeroed) or off."""
    check(load(require_gpu=True).dpf_hip_clock_probe(1 if on else 0))


def clock_probe_read() -> dict:
    """Sustained shader clock (GHz) of the octet expand launches since the
    last read, from s_memtime / s_memrealtime stamps of every workgroup."""
    ghz, wg, mean_s = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    check(load().dpf_hip_clock_probe_read(ctypes.byref(ghz), ctypes.byref(wg), ctypes.byref(mean_s)))
    return {"clock_ghz": ghz.value, "workgroups": wg.value, "mean_workgroup_ms": mean_s.value * 1e3}


def check(st: int):
    if st != 0:
        raise DpfHipError(st, load().dpf_hip_last_error().decode())


def aes_key(k: int) -> AesKey:
    a = AesKey()
    for i, b in enumerate((k & ((1 << 128) - 1)).to_bytes(16, "little")):
        a.bytes[i] = b
    return a


def value_desc(leaves: Sequence[tuple], direct: bool, elements_per_block: int,
               blocks_needed: int) -> ValueDesc:
    """leaves: [(kind, bits, modulus)]."""
    d = ValueDesc()
    d.num_leaves = len(leaves)
    d.direct = 1 if direct else 0
    d.elements_per_block = elements_per_block
    d.blocks_needed = blocks_needed
    for i, (kind, bits, mod) in enumerate(leaves):
        d.kind[i] = kind
        d.bits[i] = bits
        d.mod_low[i] = mod & MASK64
        d.mod_high[i] = (mod >> 64) & MASK64
    return d


def _p(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _stream(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def to_device_blocks(a: np.ndarray, device="cuda"):
    """numpy uint64 (n, 2) -> torch int64 tensor (n, 2) on device (same bytes)."""
    import torch
    a = np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 2)
    return torch.from_numpy(a.view(np.int64)).to(device)


def to_device_u8(a, device="cuda"):
    import torch
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return torch.from_numpy(a).to(device)


def blocks_to_numpy(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64).reshape(-1, 2)


def hash_blocks(blocks, key: int, out=None, stream=None):
    import torch
    L = load(require_gpu=True)
    n = blocks.shape[0]
    if out is None:
        out = torch.empty_like(blocks)
    k = aes_key(key)
    check(L.dpf_hip_hash(n, _p(blocks), ctypes.byref(k), _p(out), _stream(stream)))
    return out


def eval_paths(seeds, ctrl, paths, cw_seed, cw_left, cw_right, key_left: int, key_right: int,
               seeds_out=None, ctrl_out=None, stream=None):
    import torch
    L = load(require_gpu=True)
    n = seeds.shape[0]
    levels = cw_left.shape[0]
    if seeds_out is None:
        seeds_out = torch.empty_like(seeds)
    if ctrl_out is None:
        ctrl_out = torch.empty_like(ctrl)
    kl, kr = aes_key(key_left), aes_key(key_right)
    check(L.dpf_hip_eval_paths(n, levels, _p(seeds), _p(ctrl), _p(paths), _p(cw_seed),
                               _p(cw_left), _p(cw_right), ctypes.byref(kl), ctypes.byref(kr),
                               _p(seeds_out), _p(ctrl_out), _stream(stream)))
    return seeds_out, ctrl_out


def expand(seeds, ctrl, cw_seed, cw_left, cw_right, keys, desc: ValueDesc, elements_per_leaf: int,
           value_correction, party: int, out=None, stream=None):
    """Fused ExpandSeeds + HashExpandedSeeds + correction; returns packed uint8 tensor."""
    import torch
    L = load(require_gpu=True)
    n0 = seeds.shape[0]
    levels = cw_left.shape[0]
    esz = L.dpf_hip_packed_element_size(ctypes.byref(desc))
    total = (n0 << levels) * elements_per_leaf
    if out is None:
        out = torch.empty(total * esz, dtype=torch.uint8, device=seeds.device)
    kl, kr, kv = (aes_key(k) for k in keys)
    check(L.dpf_hip_expand(n0, _p(seeds), _p(ctrl), levels, _p(cw_seed), _p(cw_left),
                           _p(cw_right), ctypes.byref(kl), ctypes.byref(kr), ctypes.byref(kv),
                           ctypes.byref(desc), elements_per_leaf, _p(value_correction), party,
                           _p(out), _stream(stream)))
    return out


def eval_points(n, points_per_key, levels, key_seed, party, tree_index, block_index, cw_seed,
                cw_left, cw_right, keys, desc: ValueDesc, value_correction, seeds_in=None,
                ctrl_in=None, out=None, stream=None):
    import torch
    L = load(require_gpu=True)
    esz = L.dpf_hip_packed_element_size(ctypes.byref(desc))
    if out is None:
        out = torch.empty(max(n * esz, 1), dtype=torch.uint8, device=tree_index.device)
    kl, kr, kv = (aes_key(k) for k in keys)
    check(L.dpf_hip_eval_points(n, points_per_key, levels, _p(key_seed), _p(party), _p(seeds_in),
                                _p(ctrl_in), _p(tree_index), _p(block_index), _p(cw_seed),
                                _p(cw_left), _p(cw_right), ctypes.byref(kl), ctypes.byref(kr),
                                ctypes.byref(kv), ctypes.byref(desc), _p(value_correction),
                                _p(out), _stream(stream)))
    return out


class Event:
    """hipEvent on an explicit stream (torch.cuda.Event only sees torch's stream)."""

    def __init__(self):
        self.ev = ctypes.c_void_p()
        check(load().dpf_hip_event_create(ctypes.byref(self.ev)))

    def record(self, stream=None):
        check(load().dpf_hip_event_record(self.ev, _stream(stream)))

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        check(load().dpf_hip_event_elapsed_ms(self.ev, end.ev, ctypes.byref(ms)))
        return float(ms.value)

    def __del__(self):
        try:
            if _lib is not None and self.ev:
                _lib.dpf_hip_event_destroy(self.ev)
        except Exception:
            pass
