// proto.cc -- proto3 binary wire format for the DPF messages
// (dpf/distributed_point_function.proto:25-171).  Field numbers and wire types
// follow the .proto exactly; serialisation is in field-number order with
// proto3 implicit presence (zero scalars omitted, set oneof members and present
// sub-messages always written), which is byte-identical to the canonical
// protobuf serialisation for these messages.  Unknown fields are skipped.
#include <cmath>
#include <cstring>
#include <sstream>

#include "dpf/distributed_point_function.pb.h"
#include "dcf/distributed_comparison_function.pb.h"

namespace distributed_point_functions {
namespace {

enum WireType { kVarint = 0, kFixed64 = 1, kLen = 2, kFixed32 = 5 };

// ---------------------------------------------------------------- writing
struct Writer {
  std::string* out;
  void varint(uint64_t v) {
    while (v >= 0x80) { out->push_back(static_cast<char>((v & 0x7f) | 0x80)); v >>= 7; }
    out->push_back(static_cast<char>(v));
  }
  void tag(int field, WireType wt) { varint((static_cast<uint64_t>(field) << 3) | wt); }
  void u64(int field, uint64_t v, bool always = false) {
    if (v || always) { tag(field, kVarint); varint(v); }
  }
  void i32(int field, int32_t v) {
    if (v) { tag(field, kVarint); varint(static_cast<uint64_t>(static_cast<int64_t>(v))); }
  }
  void boolean(int field, bool v) { if (v) { tag(field, kVarint); varint(1); } }
  void dbl(int field, double v) {
    if (v != 0.0 || std::signbit(v)) {
      tag(field, kFixed64);
      uint64_t bits;
      std::memcpy(&bits, &v, 8);
      for (int i = 0; i < 8; ++i) out->push_back(static_cast<char>(bits >> (8 * i)));
    }
  }
  template <typename M>
  void msg(int field, const M& m) {
    std::string sub;
    m.SerializeToString(&sub);
    tag(field, kLen);
    varint(sub.size());
    out->append(sub);
  }
};

// ---------------------------------------------------------------- reading
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 70; s += 7) {
      if (p >= end) { ok = false; return 0; }
      uint8_t b = *p++;
      v |= static_cast<uint64_t>(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  uint64_t fixed64() {
    if (end - p < 8) { ok = false; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= static_cast<uint64_t>(p[i]) << (8 * i);
    p += 8;
    return v;
  }
  // Returns the sub-range of a length-delimited field.
  Reader len() {
    uint64_t n = varint();
    if (!ok || static_cast<uint64_t>(end - p) < n) { ok = false; return Reader{p, p, false}; }
    Reader r{p, p + n};
    p += n;
    return r;
  }
  void skip(int wt) {
    switch (wt) {
      case kVarint: varint(); break;
      case kFixed64: if (end - p < 8) ok = false; else p += 8; break;
      case kLen: len(); break;
      case kFixed32: if (end - p < 4) ok = false; else p += 4; break;
      default: ok = false;
    }
  }
};

// Nesting limit of sub-message parses: protobuf's default recursion limit.
// Value and ValueType nest through their tuples without bound, and keys come
// from untrusted clients, so deeper input is a parse error, not a stack overflow.
constexpr int kRecursionLimit = 100;
thread_local int g_depth = 0;
thread_local bool g_merge = false;

// First statement of every ParseFromArray: a top-level parse replaces the
// message; a nested one (a sub-message field, via ParseSub) merges into the
// field's current value, as protobuf does when a singular message field
// occurs more than once on the wire.
template <typename M>
void BeginParse(M* m) {
  if (g_merge) g_merge = false;
  else *m = M();
}

template <typename M>
bool ParseSub(Reader r, M* m) {
  if (!r.ok || g_depth >= kRecursionLimit) return false;
  ++g_depth;
  g_merge = true;
  const bool ok = m->ParseFromArray(r.p, static_cast<int>(r.end - r.p));
  g_merge = false;
  --g_depth;
  return ok;
}

// Parses a message body: `field(num, wt, reader)` returns false on error.
template <typename F>
bool ParseFields(const void* data, int size, F field) {
  Reader r{static_cast<const uint8_t*>(data), static_cast<const uint8_t*>(data) + size};
  while (r.ok && !r.done()) {
    uint64_t t = r.varint();
    if (!r.ok) return false;
    int num = static_cast<int>(t >> 3), wt = static_cast<int>(t & 7);
    if (num == 0) return false;
    if (!field(num, wt, r)) return false;
  }
  return r.ok;
}

// ---------------------------------------------------------------- text
struct Text {
  std::ostringstream os;
  int indent = 0;
  void pad() { for (int i = 0; i < indent; ++i) os << "  "; }
  void scalar(const char* name, const std::string& v) { pad(); os << name << ": " << v << "\n"; }
  template <typename M>
  void msg(const char* name, const M& m) {
    pad();
    os << name << " {\n";
    std::string inner = m.DebugString();
    std::istringstream is(inner);
    std::string line;
    while (std::getline(is, line)) { pad(); os << "  " << line << "\n"; }
    pad();
    os << "}\n";
  }
};

std::string FormatDouble(double v) {
  std::ostringstream os;
  os.precision(17);
  os << v;
  return os.str();
}

}  // namespace

// ============================================================== Block
bool Block::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  w.u64(1, high_);
  w.u64(2, low_);
  return true;
}
bool Block::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kVarint) high_ = r.varint();
    else if (f == 2 && wt == kVarint) low_ = r.varint();
    else r.skip(wt);
    return r.ok;
  });
}
std::string Block::DebugString() const {
  Text t;
  if (high_) t.scalar("high", std::to_string(high_));
  if (low_) t.scalar("low", std::to_string(low_));
  return t.os.str();
}
bool Block::operator==(const Block& o) const { return high_ == o.high_ && low_ == o.low_; }

// ============================================================== Value.Integer
bool Value_Integer::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (case_ == kValueUint64) w.u64(1, u64_, /*always=*/true);
  if (case_ == kValueUint128) w.msg(2, u128_);
  return true;
}
bool Value_Integer::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kVarint) set_value_uint64(r.varint());
    else if (f == 2 && wt == kLen) return ParseSub(r.len(), mutable_value_uint128());
    else r.skip(wt);
    return r.ok;
  });
}
std::string Value_Integer::DebugString() const {
  Text t;
  if (case_ == kValueUint64) t.scalar("value_uint64", std::to_string(u64_));
  if (case_ == kValueUint128) t.msg("value_uint128", u128_);
  return t.os.str();
}
bool Value_Integer::operator==(const Value_Integer& o) const {
  return case_ == o.case_ && u64_ == o.u64_ && u128_ == o.u128_;
}

// ============================================================== Value.Tuple
bool Value_Tuple::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  for (const Value& v : elements_) w.msg(1, v);
  return true;
}
bool Value_Tuple::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), add_elements());
    r.skip(wt);
    return r.ok;
  });
}
std::string Value_Tuple::DebugString() const {
  Text t;
  for (const Value& v : elements_) t.msg("elements", v);
  return t.os.str();
}
bool Value_Tuple::operator==(const Value_Tuple& o) const { return elements_ == o.elements_; }

// ============================================================== Value
bool Value::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  switch (case_) {
    case kInteger: w.msg(1, int_); break;
    case kTuple: w.msg(2, tuple_); break;
    case kIntModN: w.msg(3, int_); break;
    case kXorWrapper: w.msg(4, int_); break;
    default: break;
  }
  return true;
}
bool Value::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (wt == kLen && f >= 1 && f <= 4) {
      Reader sub = r.len();
      switch (f) {
        case 1: return ParseSub(sub, mutable_integer());
        case 2: return ParseSub(sub, mutable_tuple());
        case 3: return ParseSub(sub, mutable_int_mod_n());
        default: return ParseSub(sub, mutable_xor_wrapper());
      }
    }
    r.skip(wt);
    return r.ok;
  });
}
std::string Value::DebugString() const {
  Text t;
  switch (case_) {
    case kInteger: t.msg("integer", int_); break;
    case kTuple: t.msg("tuple", tuple_); break;
    case kIntModN: t.msg("int_mod_n", int_); break;
    case kXorWrapper: t.msg("xor_wrapper", int_); break;
    default: break;
  }
  return t.os.str();
}
bool Value::operator==(const Value& o) const {
  if (case_ != o.case_) return false;
  if (case_ == kTuple) return tuple_ == o.tuple_;
  return int_ == o.int_;
}

// ============================================================== ValueType.*
bool ValueType_Integer::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  w.i32(1, bitsize_);
  return true;
}
bool ValueType_Integer::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kVarint) bitsize_ = static_cast<int32_t>(r.varint());
    else r.skip(wt);
    return r.ok;
  });
}
std::string ValueType_Integer::DebugString() const {
  Text t;
  if (bitsize_) t.scalar("bitsize", std::to_string(bitsize_));
  return t.os.str();
}
bool ValueType_Integer::operator==(const ValueType_Integer& o) const {
  return bitsize_ == o.bitsize_;
}

bool ValueType_Tuple::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  for (const ValueType& v : elements_) w.msg(1, v);
  return true;
}
bool ValueType_Tuple::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), add_elements());
    r.skip(wt);
    return r.ok;
  });
}
std::string ValueType_Tuple::DebugString() const {
  Text t;
  for (const ValueType& v : elements_) t.msg("elements", v);
  return t.os.str();
}
bool ValueType_Tuple::operator==(const ValueType_Tuple& o) const {
  return elements_ == o.elements_;
}

bool ValueType_IntModN::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (has_base_) w.msg(1, base_);
  if (has_mod_) w.msg(2, mod_);
  return true;
}
bool ValueType_IntModN::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), mutable_base_integer());
    if (f == 2 && wt == kLen) return ParseSub(r.len(), mutable_modulus());
    r.skip(wt);
    return r.ok;
  });
}
std::string ValueType_IntModN::DebugString() const {
  Text t;
  if (has_base_) t.msg("base_integer", base_);
  if (has_mod_) t.msg("modulus", mod_);
  return t.os.str();
}
bool ValueType_IntModN::operator==(const ValueType_IntModN& o) const {
  return has_base_ == o.has_base_ && has_mod_ == o.has_mod_ && base_ == o.base_ && mod_ == o.mod_;
}

bool ValueType::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  switch (case_) {
    case kInteger: w.msg(1, int_); break;
    case kTuple: w.msg(2, tuple_); break;
    case kIntModN: w.msg(3, mod_); break;
    case kXorWrapper: w.msg(4, int_); break;
    default: break;
  }
  return true;
}
bool ValueType::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (wt == kLen && f >= 1 && f <= 4) {
      Reader sub = r.len();
      switch (f) {
        case 1: return ParseSub(sub, mutable_integer());
        case 2: return ParseSub(sub, mutable_tuple());
        case 3: return ParseSub(sub, mutable_int_mod_n());
        default: return ParseSub(sub, mutable_xor_wrapper());
      }
    }
    r.skip(wt);
    return r.ok;
  });
}
std::string ValueType::DebugString() const {
  Text t;
  switch (case_) {
    case kInteger: t.msg("integer", int_); break;
    case kTuple: t.msg("tuple", tuple_); break;
    case kIntModN: t.msg("int_mod_n", mod_); break;
    case kXorWrapper: t.msg("xor_wrapper", int_); break;
    default: break;
  }
  return t.os.str();
}
bool ValueType::operator==(const ValueType& o) const {
  if (case_ != o.case_) return false;
  if (case_ == kTuple) return tuple_ == o.tuple_;
  if (case_ == kIntModN) return mod_ == o.mod_;
  return int_ == o.int_;
}

// ============================================================== DpfParameters
bool DpfParameters::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  w.i32(1, log_domain_size_);
  if (has_vt_) w.msg(3, vt_);
  w.dbl(4, security_parameter_);
  return true;
}
bool DpfParameters::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kVarint) log_domain_size_ = static_cast<int32_t>(r.varint());
    else if (f == 3 && wt == kLen) return ParseSub(r.len(), mutable_value_type());
    else if (f == 4 && wt == kFixed64) {
      uint64_t bits = r.fixed64();
      std::memcpy(&security_parameter_, &bits, 8);
    } else r.skip(wt);
    return r.ok;
  });
}
std::string DpfParameters::DebugString() const {
  Text t;
  if (log_domain_size_) t.scalar("log_domain_size", std::to_string(log_domain_size_));
  if (has_vt_) t.msg("value_type", vt_);
  if (security_parameter_ != 0) t.scalar("security_parameter", FormatDouble(security_parameter_));
  return t.os.str();
}
bool DpfParameters::operator==(const DpfParameters& o) const {
  return log_domain_size_ == o.log_domain_size_ && has_vt_ == o.has_vt_ && vt_ == o.vt_ &&
         security_parameter_ == o.security_parameter_;
}

// ============================================================== CorrectionWord
bool CorrectionWord::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (has_seed_) w.msg(1, seed_);
  w.boolean(2, control_left_);
  w.boolean(3, control_right_);
  for (const Value& v : vc_) w.msg(5, v);
  return true;
}
bool CorrectionWord::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), mutable_seed());
    if (f == 2 && wt == kVarint) control_left_ = r.varint() != 0;
    else if (f == 3 && wt == kVarint) control_right_ = r.varint() != 0;
    else if (f == 5 && wt == kLen) return ParseSub(r.len(), add_value_correction());
    else r.skip(wt);
    return r.ok;
  });
}
std::string CorrectionWord::DebugString() const {
  Text t;
  if (has_seed_) t.msg("seed", seed_);
  if (control_left_) t.scalar("control_left", "true");
  if (control_right_) t.scalar("control_right", "true");
  for (const Value& v : vc_) t.msg("value_correction", v);
  return t.os.str();
}
bool CorrectionWord::operator==(const CorrectionWord& o) const {
  return has_seed_ == o.has_seed_ && seed_ == o.seed_ && control_left_ == o.control_left_ &&
         control_right_ == o.control_right_ && vc_ == o.vc_;
}

// ============================================================== DpfKey
bool DpfKey::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (has_seed_) w.msg(1, seed_);
  for (const CorrectionWord& c : cws_) w.msg(2, c);
  w.i32(3, party_);
  for (const Value& v : last_) w.msg(5, v);
  return true;
}
bool DpfKey::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), mutable_seed());
    if (f == 2 && wt == kLen) return ParseSub(r.len(), add_correction_words());
    if (f == 3 && wt == kVarint) party_ = static_cast<int32_t>(r.varint());
    else if (f == 5 && wt == kLen) return ParseSub(r.len(), add_last_level_value_correction());
    else r.skip(wt);
    return r.ok;
  });
}
std::string DpfKey::DebugString() const {
  Text t;
  if (has_seed_) t.msg("seed", seed_);
  for (const CorrectionWord& c : cws_) t.msg("correction_words", c);
  if (party_) t.scalar("party", std::to_string(party_));
  for (const Value& v : last_) t.msg("last_level_value_correction", v);
  return t.os.str();
}
bool DpfKey::operator==(const DpfKey& o) const {
  return has_seed_ == o.has_seed_ && seed_ == o.seed_ && cws_ == o.cws_ && party_ == o.party_ &&
         last_ == o.last_;
}

// ============================================================== PartialEvaluation
bool PartialEvaluation::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (has_prefix_) w.msg(1, prefix_);
  if (has_seed_) w.msg(2, seed_);
  w.boolean(3, control_bit_);
  return true;
}
bool PartialEvaluation::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), mutable_prefix());
    if (f == 2 && wt == kLen) return ParseSub(r.len(), mutable_seed());
    if (f == 3 && wt == kVarint) control_bit_ = r.varint() != 0;
    else r.skip(wt);
    return r.ok;
  });
}
std::string PartialEvaluation::DebugString() const {
  Text t;
  if (has_prefix_) t.msg("prefix", prefix_);
  if (has_seed_) t.msg("seed", seed_);
  if (control_bit_) t.scalar("control_bit", "true");
  return t.os.str();
}
bool PartialEvaluation::operator==(const PartialEvaluation& o) const {
  return has_prefix_ == o.has_prefix_ && has_seed_ == o.has_seed_ && prefix_ == o.prefix_ &&
         seed_ == o.seed_ && control_bit_ == o.control_bit_;
}

// ============================================================== EvaluationContext
bool EvaluationContext::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  for (const DpfParameters& p : params_) w.msg(1, p);
  if (has_key_) w.msg(2, key_);
  w.i32(3, prev_);
  for (const PartialEvaluation& p : partials_) w.msg(4, p);
  w.i32(5, partials_level_);
  return true;
}
bool EvaluationContext::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), add_parameters());
    if (f == 2 && wt == kLen) return ParseSub(r.len(), mutable_key());
    if (f == 3 && wt == kVarint) prev_ = static_cast<int32_t>(r.varint());
    else if (f == 4 && wt == kLen) return ParseSub(r.len(), add_partial_evaluations());
    else if (f == 5 && wt == kVarint) partials_level_ = static_cast<int32_t>(r.varint());
    else r.skip(wt);
    return r.ok;
  });
}
std::string EvaluationContext::DebugString() const {
  Text t;
  for (const DpfParameters& p : params_) t.msg("parameters", p);
  if (has_key_) t.msg("key", key_);
  if (prev_) t.scalar("previous_hierarchy_level", std::to_string(prev_));
  for (const PartialEvaluation& p : partials_) t.msg("partial_evaluations", p);
  if (partials_level_) t.scalar("partial_evaluations_level", std::to_string(partials_level_));
  return t.os.str();
}
bool EvaluationContext::operator==(const EvaluationContext& o) const {
  return params_ == o.params_ && has_key_ == o.has_key_ && key_ == o.key_ && prev_ == o.prev_ &&
         partials_ == o.partials_ && partials_level_ == o.partials_level_;
}

// ============================================================== DCF messages
// dcf/distributed_comparison_function.proto: DcfParameters{parameters = 1},
// DcfKey{key = 1}.
bool DcfParameters::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (has_params_) w.msg(1, params_);
  return true;
}
bool DcfParameters::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), mutable_parameters());
    r.skip(wt);
    return r.ok;
  });
}
std::string DcfParameters::DebugString() const {
  Text t;
  if (has_params_) t.msg("parameters", params_);
  return t.os.str();
}
bool DcfParameters::operator==(const DcfParameters& o) const {
  return has_params_ == o.has_params_ && params_ == o.params_;
}
bool DcfKey::SerializeToString(std::string* out) const {
  out->clear();
  Writer w{out};
  if (has_key_) w.msg(1, key_);
  return true;
}
bool DcfKey::ParseFromArray(const void* d, int n) {
  BeginParse(this);
  return ParseFields(d, n, [&](int f, int wt, Reader& r) {
    if (f == 1 && wt == kLen) return ParseSub(r.len(), mutable_key());
    r.skip(wt);
    return r.ok;
  });
}
std::string DcfKey::DebugString() const {
  Text t;
  if (has_key_) t.msg("key", key_);
  return t.os.str();
}
bool DcfKey::operator==(const DcfKey& o) const { return has_key_ == o.has_key_ && key_ == o.key_; }

#define DPF_PARSE_FROM_STRING(Name) \
  bool Name::ParseFromString(const std::string& s) { \
    return ParseFromArray(s.data(), static_cast<int>(s.size())); \
  }
DPF_PARSE_FROM_STRING(Block)
DPF_PARSE_FROM_STRING(Value_Integer)
DPF_PARSE_FROM_STRING(Value_Tuple)
DPF_PARSE_FROM_STRING(Value)
DPF_PARSE_FROM_STRING(ValueType_Integer)
DPF_PARSE_FROM_STRING(ValueType_Tuple)
DPF_PARSE_FROM_STRING(ValueType_IntModN)
DPF_PARSE_FROM_STRING(ValueType)
DPF_PARSE_FROM_STRING(DpfParameters)
DPF_PARSE_FROM_STRING(CorrectionWord)
DPF_PARSE_FROM_STRING(DpfKey)
DPF_PARSE_FROM_STRING(PartialEvaluation)
DPF_PARSE_FROM_STRING(EvaluationContext)
DPF_PARSE_FROM_STRING(DcfParameters)
DPF_PARSE_FROM_STRING(DcfKey)

}  // namespace distributed_point_functions
