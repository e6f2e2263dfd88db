"""Stream handling of the device entry points: work queued on a caller's
short-lived stream, the stream destroyed, then the same DistributedPointFunction
reused on another stream -- the staged-upload buffers are fenced with events,
never with the caller's stream (host_util.h HostStaging / PackedUploads)."""
import gc

import numpy as np
import pytest

from distributed_point_functions_amd import dpf as D
from distributed_point_functions_amd import proto as pb

pytestmark = pytest.mark.gpu


def test_destroyed_caller_stream_then_reuse():
    import torch
    p = pb.DpfParameters()
    p.log_domain_size = 16
    p.value_type.CopyFrom(D.integer_type(64))
    dpf = D.DistributedPointFunction.create(p)
    k0, k1 = dpf.generate_keys_incremental(12345, [D.to_value(D.integer_type(64), 77)],
                                           seeds=(11, 22))
    want = dpf.evaluate_until(0, [], dpf.create_evaluation_context(k0))
    out = torch.empty(1 << 16, dtype=torch.int64, device="cuda")
    for _ in range(3):
        s = torch.cuda.Stream()
        assert dpf.evaluate_until_to_device(0, [], dpf.create_evaluation_context(k0), out,
                                            stream=s) == 1 << 16
        s.synchronize()
        del s
        gc.collect()
        got = dpf.evaluate_until(0, [], dpf.create_evaluation_context(k0))   # default stream
        assert np.array_equal(np.asarray(got), np.asarray(want))
        assert np.array_equal(out.cpu().numpy().view(np.uint64), np.asarray(want).view(np.uint64))
    # Host EvaluateAt after the caller stream is gone.
    pts = [0, 12345, 65535]
    a = dpf.evaluate_at(k0, 0, pts)
    b = dpf.evaluate_at(k1, 0, pts)
    assert [(int(x) + int(y)) % (1 << 64) for x, y in zip(a, b)] == [0, 77, 0]


def test_sum_workspace_across_streams():
    """Back-to-back EvaluateAtBatchSumToDevice calls on two streams share one
    workspace of 192-bit accumulators: the second call waits for the first's
    kernels (StreamFence) instead of zeroing the workspace under them."""
    import torch
    p = pb.DpfParameters()
    p.log_domain_size = 20
    p.value_type.CopyFrom(D.integer_type(64))
    dpf = D.DistributedPointFunction.create(p)
    rng = np.random.default_rng(9)
    n_keys, n_pts = 4096, 2048
    alphas = [int(a) for a in rng.integers(0, 1 << 20, size=n_keys)]
    b0, b1 = dpf.generate_key_batch(alphas, [D.to_value(D.integer_type(64), 1)],
                                    root_seeds=rng.integers(0, 2**64, size=(2 * n_keys, 2),
                                                            dtype=np.uint64), threads=4)
    pts = np.array([[a, 0] for a in alphas[:n_pts]], np.uint64)
    points = torch.from_numpy(pts.view(np.int64)).cuda()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    d0 = dpf.upload_key_batch(b0, stream=sa)
    d1 = dpf.upload_key_batch(b1, stream=sb)
    torch.cuda.synchronize()
    outs = [torch.empty(n_pts * 8, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for _ in range(3):
        dpf.evaluate_at_batch_sum_to_device(d0, 0, points, outs[0], stream=sa)
        dpf.evaluate_at_batch_sum_to_device(d1, 0, points, outs[1], stream=sb)
        torch.cuda.synchronize()
        s0 = outs[0].cpu().numpy().view(np.uint64)
        s1 = outs[1].cpu().numpy().view(np.uint64)
        counts = np.bincount(np.asarray(alphas), minlength=1 << 20)
        np.testing.assert_array_equal(s0 + s1, counts[pts[:, 0].astype(np.int64)].astype(np.uint64))
