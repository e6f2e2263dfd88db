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
