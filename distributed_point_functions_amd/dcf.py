"""Python mirror of the reference's DistributedComparisonFunction
(dcf/distributed_comparison_function.h:30-105), backed by the host C++ class
of csrc/host/distributed_comparison_function.cc whose evaluation runs in the
gfx950 kernel dpf_hip_dcf_eval_batch.  Same names (snake_case), argument
meaning and errors (DpfStatusError with the reference's messages)."""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import dpf as D
from . import proto as pb


class DistributedComparisonFunction:
    """h:30-74.  Construct with create()."""

    def __init__(self, impl, parameters: pb.DcfParameters):
        self._impl = impl
        self._parameters = parameters

    @staticmethod
    def create(parameters: pb.DcfParameters) -> "DistributedComparisonFunction":
        impl = D._call(D.host().DistributedComparisonFunction.create,
                       parameters.SerializeToString())
        return DistributedComparisonFunction(impl, parameters)

    def parameters(self) -> pb.DcfParameters:
        return self._parameters

    def value_type(self) -> pb.ValueType:
        return self._parameters.parameters.value_type

    def generate_keys(self, alpha: int, beta, seed_0: Optional[int] = None,
                      seed_1: Optional[int] = None):
        """Keys for x -> beta if x < alpha else 0 (cc:79-101).  `beta` is a Value
        proto or a Python value of the DCF's value type; seeds (optional) make
        the keys reproducible."""
        if not isinstance(beta, pb.Value):
            beta = D.to_value(self.value_type(), beta)
        k0, k1 = D._call(self._impl.generate_keys, int(alpha), beta.SerializeToString(),
                         None if seed_0 is None else int(seed_0),
                         None if seed_1 is None else int(seed_1))
        a, b = pb.DcfKey(), pb.DcfKey()
        a.ParseFromString(k0)
        b.ParseFromString(k1)
        return a, b

    def evaluate_packed(self, key: pb.DcfKey, xs: Sequence[int],
                        value_type: Optional[pb.ValueType] = None) -> np.ndarray:
        pts = xs if isinstance(xs, np.ndarray) else D.u128_array(xs)
        out = D._call(self._impl.evaluate, key.SerializeToString(), pts,
                      None if value_type is None else value_type.SerializeToString())
        size = self._impl.packed_size()
        return out.reshape(-1, size)

    def evaluate(self, key: pb.DcfKey, x: int, value_type: Optional[pb.ValueType] = None):
        """h:83-105: the share of [x < alpha] * beta (Python int or tuple)."""
        vt = value_type if value_type is not None else self.value_type()
        return D.decode(vt, self.evaluate_packed(key, [x], value_type))[0]

    def make_key_batch(self, keys: Sequence[pb.DcfKey]):
        return D._call(self._impl.make_key_batch, [k.SerializeToString() for k in keys])

    def upload_key_batch(self, batch, begin: int = 0, end: Optional[int] = None, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        end = batch.num_keys if end is None else end
        return D._call(batch.upload, int(begin), int(end), s.cuda_stream)

    def evaluate_batch_to_device(self, device_batch, points, points_per_key: int, out,
                                 shared_points: bool = False, stream=None) -> int:
        """Evaluate for every key of a device batch at device points (torch int64
        (n, 2) {low, high}); packed [key][point] outputs in `out`."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        return D._call(self._impl.evaluate_batch_to_device, device_batch, points.data_ptr(),
                       int(points_per_key), bool(shared_points), out.data_ptr(),
                       out.numel() * out.element_size(), s.cuda_stream)

    def packed_size(self) -> int:
        return self._impl.packed_size()
