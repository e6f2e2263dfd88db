"""Host <-> device copies of the C ABI (dpf_hip_memcpy_h2d / _d2h, include/dpf_hip.h)
from several host threads at once.

Pageable copies of >= DPF_HIP_REGISTER_MIN_BYTES (512 MiB) register the host
range for the copy's duration (dpf_kernels.hip: acquire_host / release_host);
smaller ones go through the page-locked staging buffers.  Two threads copying from or
into the same range must share one reference-counted registration: the first
thread to finish must not unregister pages the other thread's DMA is still
using.  Each copy is compared byte for byte.
"""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lib():
    from distributed_point_functions_amd import hip_abi as H
    L = H.load(require_gpu=True)
    P = ctypes.c_void_p
    L.dpf_hip_memcpy_h2d.argtypes = [P, P, ctypes.c_size_t, P]
    L.dpf_hip_memcpy_d2h.argtypes = [P, P, ctypes.c_size_t, P]
    return H, L


def _threads(fns):
    errs = []

    def run(f):
        try:
            f()
        except BaseException as e:   # noqa: BLE001 -- reported below
            errs.append(e)
    ts = [threading.Thread(target=run, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


@pytest.mark.parametrize("mib,threads", [(520, 2), (1040, 3), (40, 3)])
def test_concurrent_uploads_of_one_host_buffer(mib, threads):
    import torch
    H, L = _lib()
    n = mib << 20
    src = np.random.default_rng(mib).integers(0, 2**63, size=n // 8, dtype=np.int64).view(np.uint8)
    outs = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(threads)]
    streams = [torch.cuda.Stream() for _ in range(threads)]

    def up(i):
        def f():
            for rep in range(4):
                # Overlapping sub-ranges too: the whole buffer, then its halves.
                lo, hi = [(0, n), (0, n // 2), (n // 2, n), (n // 4, 3 * n // 4)][(rep + i) % 4]
                H.check(L.dpf_hip_memcpy_h2d(outs[i].data_ptr() + lo, src.ctypes.data + lo, hi - lo,
                                             streams[i].cuda_stream))
        return f
    _threads([up(i) for i in range(threads)])
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), src)


@pytest.mark.parametrize("mib,threads", [(520, 2), (36, 4)])
def test_concurrent_downloads_into_one_host_buffer(mib, threads):
    """Every thread writes the same bytes into the same host range."""
    import torch
    H, L = _lib()
    n = mib << 20
    want = np.random.default_rng(mib + 1).integers(0, 2**63, size=n // 8, dtype=np.int64).view(np.uint8)
    dev = torch.from_numpy(want).cuda()
    dst = np.zeros(n, dtype=np.uint8)
    streams = [torch.cuda.Stream() for _ in range(threads)]

    def down(i):
        def f():
            for _ in range(3):
                H.check(L.dpf_hip_memcpy_d2h(dst.ctypes.data, dev.data_ptr(), n,
                                             streams[i].cuda_stream))
        return f
    _threads([down(i) for i in range(threads)])
    assert np.array_equal(dst, want)
