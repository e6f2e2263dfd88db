"""Python protobuf classes for the reference wire format
(dpf/distributed_point_function.proto:25-171), built from a descriptor
constructed in code (there is no protoc in this image).  Field names, numbers,
types and oneofs are those of the .proto, so the bytes interoperate with the
reference and with the C++ codec in csrc/host/proto.cc.
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
_PKG = "distributed_point_functions"


def _field(msg, name, number, ftype, label=_F.LABEL_OPTIONAL, type_name=None, oneof=None):
    f = msg.field.add()
    f.name = name
    f.number = number
    f.type = ftype
    f.label = label
    if type_name:
        f.type_name = f".{_PKG}.{type_name}"
    if oneof is not None:
        f.oneof_index = oneof
    return f


def _build():
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "dpf/distributed_point_function.proto"
    fd.package = _PKG
    fd.syntax = "proto3"
    M, R, O = _F.TYPE_MESSAGE, _F.LABEL_REPEATED, _F.LABEL_OPTIONAL

    vt = fd.message_type.add(name="ValueType")
    integer = vt.nested_type.add(name="Integer")
    _field(integer, "bitsize", 1, _F.TYPE_INT32)
    tup = vt.nested_type.add(name="Tuple")
    _field(tup, "elements", 1, M, R, "ValueType")
    imn = vt.nested_type.add(name="IntModN")
    _field(imn, "base_integer", 1, M, O, "ValueType.Integer")
    _field(imn, "modulus", 2, M, O, "Value.Integer")
    vt.oneof_decl.add(name="type")
    _field(vt, "integer", 1, M, O, "ValueType.Integer", oneof=0)
    _field(vt, "tuple", 2, M, O, "ValueType.Tuple", oneof=0)
    _field(vt, "int_mod_n", 3, M, O, "ValueType.IntModN", oneof=0)
    _field(vt, "xor_wrapper", 4, M, O, "ValueType.Integer", oneof=0)

    val = fd.message_type.add(name="Value")
    vint = val.nested_type.add(name="Integer")
    vint.oneof_decl.add(name="value")
    _field(vint, "value_uint64", 1, _F.TYPE_UINT64, oneof=0)
    _field(vint, "value_uint128", 2, M, O, "Block", oneof=0)
    vtup = val.nested_type.add(name="Tuple")
    _field(vtup, "elements", 1, M, R, "Value")
    val.oneof_decl.add(name="value")
    _field(val, "integer", 1, M, O, "Value.Integer", oneof=0)
    _field(val, "tuple", 2, M, O, "Value.Tuple", oneof=0)
    _field(val, "int_mod_n", 3, M, O, "Value.Integer", oneof=0)
    _field(val, "xor_wrapper", 4, M, O, "Value.Integer", oneof=0)

    p = fd.message_type.add(name="DpfParameters")
    _field(p, "log_domain_size", 1, _F.TYPE_INT32)
    _field(p, "value_type", 3, M, O, "ValueType")
    _field(p, "security_parameter", 4, _F.TYPE_DOUBLE)

    b = fd.message_type.add(name="Block")
    _field(b, "high", 1, _F.TYPE_UINT64)
    _field(b, "low", 2, _F.TYPE_UINT64)

    cw = fd.message_type.add(name="CorrectionWord")
    _field(cw, "seed", 1, M, O, "Block")
    _field(cw, "control_left", 2, _F.TYPE_BOOL)
    _field(cw, "control_right", 3, _F.TYPE_BOOL)
    _field(cw, "value_correction", 5, M, R, "Value")

    k = fd.message_type.add(name="DpfKey")
    _field(k, "seed", 1, M, O, "Block")
    _field(k, "correction_words", 2, M, R, "CorrectionWord")
    _field(k, "party", 3, _F.TYPE_INT32)
    _field(k, "last_level_value_correction", 5, M, R, "Value")

    pe = fd.message_type.add(name="PartialEvaluation")
    _field(pe, "prefix", 1, M, O, "Block")
    _field(pe, "seed", 2, M, O, "Block")
    _field(pe, "control_bit", 3, _F.TYPE_BOOL)

    ec = fd.message_type.add(name="EvaluationContext")
    _field(ec, "parameters", 1, M, R, "DpfParameters")
    _field(ec, "key", 2, M, O, "DpfKey")
    _field(ec, "previous_hierarchy_level", 3, _F.TYPE_INT32)
    _field(ec, "partial_evaluations", 4, M, R, "PartialEvaluation")
    _field(ec, "partial_evaluations_level", 5, _F.TYPE_INT32)

    # dcf/distributed_comparison_function.proto
    dcf = descriptor_pb2.FileDescriptorProto()
    dcf.name = "dcf/distributed_comparison_function.proto"
    dcf.package = _PKG
    dcf.syntax = "proto3"
    dcf.dependency.append(fd.name)
    dp = dcf.message_type.add(name="DcfParameters")
    _field(dp, "parameters", 1, M, O, "DpfParameters")
    dk = dcf.message_type.add(name="DcfKey")
    _field(dk, "key", 1, M, O, "DpfKey")

    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    pool.Add(dcf)
    out = {}
    for name in ("ValueType", "Value", "DpfParameters", "Block", "CorrectionWord", "DpfKey",
                 "PartialEvaluation", "EvaluationContext", "DcfParameters", "DcfKey"):
        out[name] = message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{name}"))
    return out


_CLASSES = _build()
ValueType = _CLASSES["ValueType"]
Value = _CLASSES["Value"]
DpfParameters = _CLASSES["DpfParameters"]
Block = _CLASSES["Block"]
CorrectionWord = _CLASSES["CorrectionWord"]
DpfKey = _CLASSES["DpfKey"]
PartialEvaluation = _CLASSES["PartialEvaluation"]
EvaluationContext = _CLASSES["EvaluationContext"]
DcfParameters = _CLASSES["DcfParameters"]
DcfKey = _CLASSES["DcfKey"]
