"""Python mirror of the reference's DistributedPointFunction API
(dpf/distributed_point_function.h:77-365), backed by the host C++ library
(lib/libdpf.so via the _dpf_host pybind module), whose evaluation runs in the
gfx950 kernels of lib/libdpf_hip.so.  Same method names (snake_case), argument
meaning and error behaviour: failing calls raise DpfStatusError carrying the
absl status code and the reference's message.

Outputs: evaluate_* return numpy arrays.  For single-leaf types of <= 64 bits
the array has the natural dtype (uint8/16/32/64); otherwise it is the packed
element layout, shape (n, packed_size) uint8 (leaves concatenated
little-endian); decode() turns either into Python values.
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import proto as pb

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBDIR = os.path.join(_HERE, "lib")
_host = None

STATUS_NAMES = {0: "OK", 3: "INVALID_ARGUMENT", 8: "RESOURCE_EXHAUSTED", 9: "FAILED_PRECONDITION",
                12: "UNIMPLEMENTED", 13: "INTERNAL", 11: "OUT_OF_RANGE", 5: "NOT_FOUND"}
MASK64 = (1 << 64) - 1


class DpfStatusError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {message}")
        self.code = code
        self.code_name = STATUS_NAMES.get(code, str(code))
        self.message = message


def host():
    """Loads the pybind module (after torch, so one HIP runtime is shared)."""
    global _host
    if _host is None:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if _LIBDIR not in sys.path:
            sys.path.insert(0, _LIBDIR)
        try:
            import _dpf_host  # noqa: F401
        except ImportError as e:
            raise DpfStatusError(13, f"host library not built ({e}); run "
                                     "python -m distributed_point_functions_amd.build_native")
        _host = _dpf_host
    return _host


def _call(fn, *args):
    try:
        return fn(*args)
    except host().StatusError as e:
        code, _, msg = str(e).partition("|")
        raise DpfStatusError(int(code), msg) from None


def u128_from_block(b) -> int:
    """Python int of a proto Block {high, low}."""
    return (int(b.high) << 64) | int(b.low)


def u128_array(xs: Sequence[int]) -> np.ndarray:
    a = np.empty((len(xs), 2), dtype=np.uint64)
    for i, x in enumerate(xs):
        x = int(x)
        a[i, 0] = x & MASK64
        a[i, 1] = (x >> 64) & MASK64
    return a


# ---------------------------------------------------------------- value types
def integer_type(bits: int) -> pb.ValueType:
    vt = pb.ValueType()
    vt.integer.bitsize = bits
    return vt


def xor_wrapper_type(bits: int) -> pb.ValueType:
    vt = pb.ValueType()
    vt.xor_wrapper.bitsize = bits
    return vt


def int_mod_n_type(base_bits: int, modulus: int) -> pb.ValueType:
    vt = pb.ValueType()
    vt.int_mod_n.base_integer.bitsize = base_bits
    _set_integer(vt.int_mod_n.modulus, modulus)
    return vt


def tuple_type(*elements: pb.ValueType) -> pb.ValueType:
    vt = pb.ValueType()
    vt.tuple.SetInParent()
    for e in elements:
        vt.tuple.elements.add().CopyFrom(e)
    return vt


def _set_integer(msg, v: int):
    # Uint128ToValueInteger (value_type_helpers.cc:134-144)
    v = int(v)
    if v >> 64 == 0:
        msg.value_uint64 = v
    else:
        msg.value_uint128.high = v >> 64
        msg.value_uint128.low = v & MASK64


def _get_integer(msg) -> int:
    which = msg.WhichOneof("value")
    if which == "value_uint128":
        return (msg.value_uint128.high << 64) | msg.value_uint128.low
    return msg.value_uint64


def to_value(vt: pb.ValueType, x) -> pb.Value:
    """ToValue for a runtime ValueType: ints for leaves, sequences for tuples."""
    v = pb.Value()
    kind = vt.WhichOneof("type")
    if kind == "integer":
        _set_integer(v.integer, x)
    elif kind == "int_mod_n":
        _set_integer(v.int_mod_n, x)
    elif kind == "xor_wrapper":
        _set_integer(v.xor_wrapper, x)
    elif kind == "tuple":
        v.tuple.SetInParent()
        for et, ex in zip(vt.tuple.elements, x):
            v.tuple.elements.add().CopyFrom(to_value(et, ex))
    else:
        raise ValueError("unsupported value type")
    return v


def from_value(vt: pb.ValueType, v: pb.Value):
    kind = vt.WhichOneof("type")
    if kind == "tuple":
        return tuple(from_value(et, ev) for et, ev in zip(vt.tuple.elements, v.tuple.elements))
    return _get_integer(getattr(v, kind))


def leaves_of(vt: pb.ValueType) -> List[Tuple[str, int, int]]:
    kind = vt.WhichOneof("type")
    if kind == "integer":
        return [("int", vt.integer.bitsize, 0)]
    if kind == "xor_wrapper":
        return [("xor", vt.xor_wrapper.bitsize, 0)]
    if kind == "int_mod_n":
        return [("intmodn", vt.int_mod_n.base_integer.bitsize, _get_integer(vt.int_mod_n.modulus))]
    out = []
    for e in vt.tuple.elements:
        out += leaves_of(e)
    return out


def decode(vt: pb.ValueType, arr: np.ndarray) -> list:
    """Packed or natural-dtype output -> list of Python values (nested tuples)."""
    ls = leaves_of(vt)
    size = sum(b // 8 for _, b, _ in ls)
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1, size)
    out = []
    for row in raw:
        b = row.tobytes()
        vals, off = [], 0
        for _, bits, _ in ls:
            vals.append(int.from_bytes(b[off:off + bits // 8], "little"))
            off += bits // 8
        it = iter(vals)
        out.append(_rebuild(vt, it))
    return out


def _rebuild(vt, it):
    if vt.WhichOneof("type") == "tuple":
        return tuple(_rebuild(e, it) for e in vt.tuple.elements)
    return next(it)


def _natural(vt: pb.ValueType, packed: np.ndarray, n: int) -> np.ndarray:
    ls = leaves_of(vt)
    size = sum(b // 8 for _, b, _ in ls)
    packed = packed.reshape(n, size) if n else packed.reshape(0, size)
    if len(ls) == 1 and ls[0][1] <= 64:
        return packed.view({8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}[ls[0][1]]).reshape(-1)
    return packed


class DistributedPointFunction:
    """h:77-365.  Construct with create() / create_incremental()."""

    def __init__(self, impl, parameters: List[pb.DpfParameters]):
        self._impl = impl
        self._parameters = parameters

    @staticmethod
    def create(parameters: pb.DpfParameters) -> "DistributedPointFunction":
        return DistributedPointFunction.create_incremental([parameters])

    @staticmethod
    def create_incremental(parameters: Sequence[pb.DpfParameters]) -> "DistributedPointFunction":
        impl = _call(host().DistributedPointFunction.create_incremental,
                     [p.SerializeToString() for p in parameters])
        params = []
        for b in impl.parameters():
            p = pb.DpfParameters()
            p.ParseFromString(b)
            params.append(p)
        return DistributedPointFunction(impl, params)

    def parameters(self) -> List[pb.DpfParameters]:
        return list(self._parameters)

    def register_value_type(self, value_type: pb.ValueType) -> None:
        _call(self._impl.register_value_type, value_type.SerializeToString())

    def to_value(self, value_type: pb.ValueType, x) -> pb.Value:
        self.register_value_type(value_type)
        return to_value(value_type, x)

    # -- key generation (CPU) ------------------------------------------------
    def _betas(self, beta) -> List[bytes]:
        out = []
        for b in beta:
            if isinstance(b, pb.Value):
                out.append(b.SerializeToString())
            else:  # plain integer (uint128 overload, h:160-164)
                out.append(to_value(integer_type(128), b).SerializeToString())
        return out

    def generate_keys(self, alpha: int, beta) -> Tuple[pb.DpfKey, pb.DpfKey]:
        return self.generate_keys_incremental(alpha, [beta])

    def generate_keys_incremental(self, alpha: int, beta: Sequence,
                                  seeds: Optional[Tuple[int, int]] = None):
        if seeds is None:
            a, b = _call(self._impl.generate_keys_incremental, int(alpha), self._betas(beta))
        else:
            a, b = _call(self._impl.generate_keys_incremental_with_seeds, int(alpha),
                         self._betas(beta), int(seeds[0]), int(seeds[1]))
        k0, k1 = pb.DpfKey(), pb.DpfKey()
        k0.ParseFromString(a)
        k1.ParseFromString(b)
        return k0, k1

    def create_evaluation_context(self, key: pb.DpfKey) -> pb.EvaluationContext:
        ctx = pb.EvaluationContext()
        ctx.ParseFromString(_call(self._impl.create_evaluation_context, key.SerializeToString()))
        return ctx

    # -- evaluation (GPU) ----------------------------------------------------
    def _type(self, h, value_type):
        if value_type is not None:
            return value_type
        return self._parameters[h].value_type if 0 <= h < len(self._parameters) else None

    def evaluate_until(self, hierarchy_level: int, prefixes: Sequence[int],
                       ctx: pb.EvaluationContext, value_type: Optional[pb.ValueType] = None,
                       packed: bool = False) -> np.ndarray:
        vt_bytes = value_type.SerializeToString() if value_type is not None else None
        out, new_ctx = _call(self._impl.evaluate_until, int(hierarchy_level), u128_array(prefixes),
                             ctx.SerializeToString(), vt_bytes)
        ctx.ParseFromString(new_ctx)
        vt = self._type(hierarchy_level, value_type)
        size = sum(b // 8 for _, b, _ in leaves_of(vt))
        n = out.size // size
        return out.reshape(n, size) if packed else _natural(vt, out, n)

    def evaluate_next(self, prefixes: Sequence[int], ctx: pb.EvaluationContext, **kw):
        if len(prefixes) == 0:
            return self.evaluate_until(0, prefixes, ctx, **kw)
        return self.evaluate_until(ctx.previous_hierarchy_level + 1, prefixes, ctx, **kw)

    def evaluate_at(self, key_or_level, level_or_points, points=None, ctx=None,
                    value_type: Optional[pb.ValueType] = None, packed: bool = False):
        """evaluate_at(key, level, points)  or  evaluate_at(level, points, ctx=ctx)
        (the two overloads of h:331-360)."""
        vt_bytes = value_type.SerializeToString() if value_type is not None else None
        if isinstance(key_or_level, pb.DpfKey):
            key, h, pts = key_or_level, int(level_or_points), points
            out = _call(self._impl.evaluate_at, key.SerializeToString(), h, u128_array(pts),
                        vt_bytes)
        else:
            h, pts = int(key_or_level), level_or_points
            if ctx is None:
                ctx = points
            out, new_ctx = _call(self._impl.evaluate_at_ctx, h, u128_array(pts),
                                 ctx.SerializeToString(), vt_bytes)
            ctx.ParseFromString(new_ctx)
        vt = self._type(h, value_type)
        size = sum(b // 8 for _, b, _ in leaves_of(vt))
        n = out.size // size
        return out.reshape(n, size) if packed else _natural(vt, out, n)

    # -- MI355X extensions -----------------------------------------------------
    def evaluate_until_to_device(self, hierarchy_level: int, prefixes: Sequence[int],
                                 ctx: pb.EvaluationContext, out, stream=None) -> int:
        """Writes packed outputs into the torch device tensor `out`; returns the
        number of elements.  `stream`: a torch.cuda.Stream (default: current)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        n, new_ctx = _call(self._impl.evaluate_until_to_device, int(hierarchy_level),
                           u128_array(prefixes), ctx.SerializeToString(), out.data_ptr(),
                           out.numel() * out.element_size(), s.cuda_stream, None)
        ctx.ParseFromString(new_ctx)
        return n

    def evaluate_shard_to_device(self, hierarchy_level: int, shard: int, num_shards: int,
                                 ctx: pb.EvaluationContext, out, stream=None) -> int:
        """Full-domain evaluation of one subtree-prefix shard into device tensor `out`."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        n, new_ctx = _call(self._impl.evaluate_shard_to_device, int(hierarchy_level), int(shard),
                           int(num_shards), ctx.SerializeToString(), out.data_ptr(),
                           out.numel() * out.element_size(), s.cuda_stream)
        ctx.ParseFromString(new_ctx)
        return n

    def evaluate_at_batch(self, keys: Sequence[pb.DpfKey], hierarchy_level: int,
                          points: Sequence[int], points_per_key: int, packed: bool = False):
        pts = points if isinstance(points, np.ndarray) else u128_array(points)
        out = _call(self._impl.evaluate_at_batch, [k.SerializeToString() for k in keys],
                    int(hierarchy_level), pts, int(points_per_key))
        vt = self._parameters[hierarchy_level].value_type
        size = sum(b // 8 for _, b, _ in leaves_of(vt))
        n = out.size // size
        return out.reshape(n, size) if packed else _natural(vt, out, n)

    # -- key batches -------------------
    def make_key_batch(self, keys: Sequence[pb.DpfKey]):
        """SoA image of `keys` (host); .upload(begin, end, stream) puts rows on the GPU."""
        return _call(self._impl.make_key_batch, [k.SerializeToString() for k in keys])

    def parse_key_batch(self, serialized_keys: Sequence[bytes], threads: int = 0):
        """SoA key batch straight from serialized DpfKeys, parsed and validated
        on host threads (batched key ingestion)."""
        return _call(self._impl.parse_key_batch, list(serialized_keys), int(threads))

    def serialize_key_batch(self, batch, threads: int = 0) -> List[bytes]:
        """Every row of a key batch as a serialized DpfKey (inverse of
        parse_key_batch), on host threads."""
        return _call(self._impl.serialize_key_batch, batch, int(threads))

    def key_from_batch(self, batch, k: int) -> pb.DpfKey:
        key = pb.DpfKey()
        key.ParseFromString(_call(self._impl.key_from_batch, batch, int(k)))
        return key

    def generate_key_batch(self, alphas: Sequence[int], beta: Sequence,
                           root_seeds: Optional[np.ndarray] = None, threads: int = 0):
        """Both parties' key batches for every alpha (shared beta per hierarchy
        level), generated on `threads` host threads.  root_seeds: uint64 (2n, 2)
        array ({low, high} per seed, two per key) or None for fresh randomness."""
        al = alphas if isinstance(alphas, np.ndarray) else u128_array(alphas)
        return _call(self._impl.generate_key_batch, al, self._betas(beta), root_seeds, int(threads))

    def upload_key_batch(self, batch, begin: int = 0, end: Optional[int] = None, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        end = batch.num_keys if end is None else end
        return _call(batch.upload, int(begin), int(end), s.cuda_stream)

    def evaluate_at_batch_to_device(self, device_batch, hierarchy_level: int, points,
                                    points_per_key: int, out, shared_points: bool = False,
                                    stream=None) -> int:
        """EvaluateAt for every key of a device batch at device points (a torch
        int64 tensor (n, 2) of {low, high}); packed outputs [key][point] in `out`."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        return _call(self._impl.evaluate_at_batch_to_device, device_batch, int(hierarchy_level),
                     points.data_ptr(), int(points_per_key), bool(shared_points), out.data_ptr(),
                     out.numel() * out.element_size(), s.cuda_stream)

    def evaluate_at_batch_sum_to_device(self, device_batch, hierarchy_level: int, points, out,
                                        stream=None) -> None:
        """out[j] = group sum over the batch's keys of EvaluateAt(key, points[j])."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        _call(self._impl.evaluate_at_batch_sum_to_device, device_batch, int(hierarchy_level),
              points.data_ptr(), int(points.shape[0]), out.data_ptr(), s.cuda_stream)

    # -- device-resident incremental evaluation of a key batch (8f.1, cfg 5b) --
    def create_batch_evaluation_context(self, device_batch):
        """EvaluationContext of every key of a device batch, kept on the GPU."""
        return _call(self._impl.create_batch_evaluation_context, device_batch)

    def evaluate_until_batch_to_device(self, hierarchy_level: int, prefixes, batch_ctx, out,
                                       sum_over_keys: bool = False, stream=None) -> int:
        """EvaluateUntil(hierarchy_level, prefixes, ctx_k) for every key k of the
        batch (same prefixes for all keys).  Packed outputs go to the torch
        device tensor `out`: [key][element], or with `sum_over_keys` the group
        sum over keys [element].  Returns the elements per key."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        pre = prefixes if isinstance(prefixes, np.ndarray) else u128_array(prefixes)
        return _call(self._impl.evaluate_until_batch_to_device, int(hierarchy_level), pre,
                     batch_ctx, bool(sum_over_keys), out.data_ptr(),
                     out.numel() * out.element_size(), s.cuda_stream)

    def evaluate_next_batch_to_device(self, prefixes, batch_ctx, out, sum_over_keys: bool = False,
                                      stream=None) -> int:
        """EvaluateNext for every key of the batch (h:363-365)."""
        level = 0 if len(prefixes) == 0 else batch_ctx.previous_hierarchy_level + 1
        return self.evaluate_until_batch_to_device(level, prefixes, batch_ctx, out,
                                                   sum_over_keys, stream)

    def export_evaluation_context(self, batch_ctx, host_batch, k: int,
                                  stream=None) -> pb.EvaluationContext:
        """Key k's context as the EvaluationContext proto EvaluateUntil leaves."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        ctx = pb.EvaluationContext()
        ctx.ParseFromString(_call(self._impl.export_evaluation_context, batch_ctx, host_batch,
                                  int(k), s.cuda_stream))
        return ctx

    def sum_packed_shares(self, hierarchy_level: int, shares: np.ndarray, num_shares: int,
                          count: int) -> np.ndarray:
        """Group sum of num_shares packed vectors of `count` elements (host)."""
        return _call(self._impl.sum_packed_shares, int(hierarchy_level),
                     np.ascontiguousarray(shares, dtype=np.uint8).reshape(-1), int(num_shares),
                     int(count))

    def packed_size(self, h: int) -> int:
        return self._impl.packed_size(h)

    def output_elements(self, h: int, num_prefixes: int, previous_hierarchy_level: int) -> int:
        """Elements EvaluateUntil(h, prefixes) returns for len(prefixes) == num_prefixes."""
        return _call(self._impl.output_elements, int(h), int(num_prefixes),
                     int(previous_hierarchy_level))

    def tree_levels_needed(self) -> int:
        return self._impl.tree_levels_needed()

    def hierarchy_to_tree(self) -> List[int]:
        return list(self._impl.hierarchy_to_tree())

    def blocks_needed(self, h: int) -> int:
        return self._impl.blocks_needed(h)
