// distributed_point_function.pb.h -- hand-written proto3 messages for the
// reference schema (dpf/distributed_point_function.proto:25-171).  There is no
// protoc/libprotobuf in this image, so the classes mirror the subset of the
// generated-code API the DPF uses, and proto.cc implements the binary wire
// format (field numbers and types exactly as the .proto), so serialized
// DpfKey / EvaluationContext bytes interoperate with any protobuf runtime.
#ifndef DPF_DISTRIBUTED_POINT_FUNCTION_PB_H_
#define DPF_DISTRIBUTED_POINT_FUNCTION_PB_H_

#include <cstdint>
#include <string>
#include <vector>

namespace distributed_point_functions {

// Repeated-field helper with the generated-code spellings used by callers.
template <typename T>
class RepeatedField {
 public:
  using value_type = T;
  int size() const { return static_cast<int>(v_.size()); }
  bool empty() const { return v_.empty(); }
  const T& operator[](int i) const { return v_[i]; }
  T& operator[](int i) { return v_[i]; }
  const T& Get(int i) const { return v_[i]; }
  T* Mutable(int i) { return &v_[i]; }
  T* Add() { v_.emplace_back(); return &v_.back(); }
  void Clear() { v_.clear(); }
  void Reserve(int n) { v_.reserve(n); }
  typename std::vector<T>::const_iterator begin() const { return v_.begin(); }
  typename std::vector<T>::const_iterator end() const { return v_.end(); }
  typename std::vector<T>::iterator begin() { return v_.begin(); }
  typename std::vector<T>::iterator end() { return v_.end(); }
  typename std::vector<T>::iterator erase(typename std::vector<T>::const_iterator it) {
    return v_.erase(it);
  }
  std::vector<T>& vec() { return v_; }
  const std::vector<T>& vec() const { return v_; }
  friend bool operator==(const RepeatedField& a, const RepeatedField& b) { return a.v_ == b.v_; }

 private:
  std::vector<T> v_;
};

// Common message base: binary (de)serialisation and text rendering.
#define DPF_PROTO_MESSAGE_API(Name)                                 \
  bool SerializeToString(std::string* out) const;                   \
  std::string SerializeAsString() const {                           \
    std::string s;                                                  \
    SerializeToString(&s);                                          \
    return s;                                                       \
  }                                                                 \
  bool ParseFromString(const std::string& data);                    \
  bool ParseFromArray(const void* data, int size);                  \
  std::string DebugString() const;                                  \
  void Clear() { *this = Name(); }                                  \
  bool operator==(const Name& o) const;                             \
  bool operator!=(const Name& o) const { return !(*this == o); }

class Block {
 public:
  uint64_t high() const { return high_; }
  uint64_t low() const { return low_; }
  void set_high(uint64_t v) { high_ = v; }
  void set_low(uint64_t v) { low_ = v; }
  DPF_PROTO_MESSAGE_API(Block)

 private:
  uint64_t high_ = 0, low_ = 0;
};

class Value;
class ValueType;

class Value_Integer {
 public:
  enum ValueCase { VALUE_NOT_SET = 0, kValueUint64 = 1, kValueUint128 = 2 };
  ValueCase value_case() const { return case_; }
  uint64_t value_uint64() const { return case_ == kValueUint64 ? u64_ : 0; }
  void set_value_uint64(uint64_t v) { case_ = kValueUint64; u64_ = v; u128_ = Block(); }
  bool has_value_uint128() const { return case_ == kValueUint128; }
  const Block& value_uint128() const;
  Block* mutable_value_uint128() { if (case_ != kValueUint128) { case_ = kValueUint128; u64_ = 0; u128_ = Block(); } return &u128_; }
  void clear_value() { case_ = VALUE_NOT_SET; u64_ = 0; u128_ = Block(); }
  DPF_PROTO_MESSAGE_API(Value_Integer)

 private:
  ValueCase case_ = VALUE_NOT_SET;
  uint64_t u64_ = 0;
  Block u128_;
};

class Value_Tuple {
 public:
  int elements_size() const { return elements_.size(); }
  const Value& elements(int i) const;
  Value* mutable_elements(int i);
  Value* add_elements();
  const RepeatedField<Value>& elements() const { return elements_; }
  RepeatedField<Value>* mutable_elements() { return &elements_; }
  DPF_PROTO_MESSAGE_API(Value_Tuple)

 private:
  RepeatedField<Value> elements_;
};

class Value {
 public:
  using Integer = Value_Integer;
  using Tuple = Value_Tuple;
  enum ValueCase { VALUE_NOT_SET = 0, kInteger = 1, kTuple = 2, kIntModN = 3, kXorWrapper = 4 };
  ValueCase value_case() const { return case_; }
  bool has_integer() const { return case_ == kInteger; }
  bool has_tuple() const { return case_ == kTuple; }
  bool has_int_mod_n() const { return case_ == kIntModN; }
  bool has_xor_wrapper() const { return case_ == kXorWrapper; }
  const Integer& integer() const;
  const Tuple& tuple() const;
  const Integer& int_mod_n() const;
  const Integer& xor_wrapper() const;
  Integer* mutable_integer() { Switch(kInteger); return &int_; }
  Tuple* mutable_tuple() { Switch(kTuple); return &tuple_; }
  Integer* mutable_int_mod_n() { Switch(kIntModN); return &int_; }
  Integer* mutable_xor_wrapper() { Switch(kXorWrapper); return &int_; }
  void clear_value() { case_ = VALUE_NOT_SET; int_ = Integer(); tuple_ = Tuple(); }
  DPF_PROTO_MESSAGE_API(Value)

 private:
  void Switch(ValueCase c) {
    if (case_ != c) { case_ = c; int_ = Integer(); tuple_ = Tuple(); }
  }
  ValueCase case_ = VALUE_NOT_SET;
  Integer int_;   // integer / int_mod_n / xor_wrapper share storage (oneof)
  Tuple tuple_;
};

class ValueType_Integer {
 public:
  int32_t bitsize() const { return bitsize_; }
  void set_bitsize(int32_t v) { bitsize_ = v; }
  DPF_PROTO_MESSAGE_API(ValueType_Integer)

 private:
  int32_t bitsize_ = 0;
};

class ValueType_Tuple {
 public:
  int elements_size() const { return elements_.size(); }
  const ValueType& elements(int i) const;
  ValueType* mutable_elements(int i);
  ValueType* add_elements();
  const RepeatedField<ValueType>& elements() const { return elements_; }
  DPF_PROTO_MESSAGE_API(ValueType_Tuple)

 private:
  RepeatedField<ValueType> elements_;
};

class ValueType_IntModN {
 public:
  bool has_base_integer() const { return has_base_; }
  const ValueType_Integer& base_integer() const { return base_; }
  ValueType_Integer* mutable_base_integer() { has_base_ = true; return &base_; }
  bool has_modulus() const { return has_mod_; }
  const Value_Integer& modulus() const { return mod_; }
  Value_Integer* mutable_modulus() { has_mod_ = true; return &mod_; }
  void clear_modulus() { has_mod_ = false; mod_ = Value_Integer(); }
  DPF_PROTO_MESSAGE_API(ValueType_IntModN)

 private:
  bool has_base_ = false, has_mod_ = false;
  ValueType_Integer base_;
  Value_Integer mod_;
};

class ValueType {
 public:
  using Integer = ValueType_Integer;
  using Tuple = ValueType_Tuple;
  using IntModN = ValueType_IntModN;
  enum TypeCase { TYPE_NOT_SET = 0, kInteger = 1, kTuple = 2, kIntModN = 3, kXorWrapper = 4 };
  TypeCase type_case() const { return case_; }
  bool has_integer() const { return case_ == kInteger; }
  bool has_tuple() const { return case_ == kTuple; }
  bool has_int_mod_n() const { return case_ == kIntModN; }
  bool has_xor_wrapper() const { return case_ == kXorWrapper; }
  const Integer& integer() const;
  const Tuple& tuple() const;
  const IntModN& int_mod_n() const;
  const Integer& xor_wrapper() const;
  Integer* mutable_integer() { Switch(kInteger); return &int_; }
  Tuple* mutable_tuple() { Switch(kTuple); return &tuple_; }
  IntModN* mutable_int_mod_n() { Switch(kIntModN); return &mod_; }
  Integer* mutable_xor_wrapper() { Switch(kXorWrapper); return &int_; }
  DPF_PROTO_MESSAGE_API(ValueType)

 private:
  void Switch(TypeCase c) {
    if (case_ != c) { case_ = c; int_ = Integer(); tuple_ = Tuple(); mod_ = IntModN(); }
  }
  TypeCase case_ = TYPE_NOT_SET;
  Integer int_;  // integer / xor_wrapper (oneof)
  Tuple tuple_;
  IntModN mod_;
};

class DpfParameters {
 public:
  int32_t log_domain_size() const { return log_domain_size_; }
  void set_log_domain_size(int32_t v) { log_domain_size_ = v; }
  bool has_value_type() const { return has_vt_; }
  const ValueType& value_type() const { return vt_; }
  ValueType* mutable_value_type() { has_vt_ = true; return &vt_; }
  void clear_value_type() { has_vt_ = false; vt_ = ValueType(); }
  double security_parameter() const { return security_parameter_; }
  void set_security_parameter(double v) { security_parameter_ = v; }
  DPF_PROTO_MESSAGE_API(DpfParameters)

 private:
  int32_t log_domain_size_ = 0;
  bool has_vt_ = false;
  ValueType vt_;
  double security_parameter_ = 0;
};

class CorrectionWord {
 public:
  bool has_seed() const { return has_seed_; }
  const Block& seed() const { return seed_; }
  Block* mutable_seed() { has_seed_ = true; return &seed_; }
  bool control_left() const { return control_left_; }
  void set_control_left(bool v) { control_left_ = v; }
  bool control_right() const { return control_right_; }
  void set_control_right(bool v) { control_right_ = v; }
  int value_correction_size() const { return vc_.size(); }
  const Value& value_correction(int i) const { return vc_[i]; }
  Value* add_value_correction() { return vc_.Add(); }
  const RepeatedField<Value>& value_correction() const { return vc_; }
  RepeatedField<Value>* mutable_value_correction() { return &vc_; }
  DPF_PROTO_MESSAGE_API(CorrectionWord)

 private:
  bool has_seed_ = false;
  Block seed_;
  bool control_left_ = false, control_right_ = false;
  RepeatedField<Value> vc_;
};

class DpfKey {
 public:
  bool has_seed() const { return has_seed_; }
  const Block& seed() const { return seed_; }
  Block* mutable_seed() { has_seed_ = true; return &seed_; }
  int correction_words_size() const { return cws_.size(); }
  const CorrectionWord& correction_words(int i) const { return cws_[i]; }
  CorrectionWord* mutable_correction_words(int i) { return cws_.Mutable(i); }
  CorrectionWord* add_correction_words() { return cws_.Add(); }
  const RepeatedField<CorrectionWord>& correction_words() const { return cws_; }
  RepeatedField<CorrectionWord>* mutable_correction_words() { return &cws_; }
  int32_t party() const { return party_; }
  void set_party(int32_t v) { party_ = v; }
  int last_level_value_correction_size() const { return last_.size(); }
  const Value& last_level_value_correction(int i) const { return last_[i]; }
  Value* add_last_level_value_correction() { return last_.Add(); }
  const RepeatedField<Value>& last_level_value_correction() const { return last_; }
  RepeatedField<Value>* mutable_last_level_value_correction() { return &last_; }
  DPF_PROTO_MESSAGE_API(DpfKey)

 private:
  bool has_seed_ = false;
  Block seed_;
  RepeatedField<CorrectionWord> cws_;
  int32_t party_ = 0;
  RepeatedField<Value> last_;
};

class PartialEvaluation {
 public:
  bool has_prefix() const { return has_prefix_; }
  const Block& prefix() const { return prefix_; }
  Block* mutable_prefix() { has_prefix_ = true; return &prefix_; }
  bool has_seed() const { return has_seed_; }
  const Block& seed() const { return seed_; }
  Block* mutable_seed() { has_seed_ = true; return &seed_; }
  bool control_bit() const { return control_bit_; }
  void set_control_bit(bool v) { control_bit_ = v; }
  DPF_PROTO_MESSAGE_API(PartialEvaluation)

 private:
  // The flags after the two blocks: 40 bytes per element instead of 48 (a
  // context holds ~1 M of these per level in config 5a, rewritten per call).
  Block prefix_, seed_;
  bool has_prefix_ = false, has_seed_ = false;
  bool control_bit_ = false;
};

class EvaluationContext {
 public:
  int parameters_size() const { return params_.size(); }
  const DpfParameters& parameters(int i) const { return params_[i]; }
  DpfParameters* add_parameters() { return params_.Add(); }
  const RepeatedField<DpfParameters>& parameters() const { return params_; }
  RepeatedField<DpfParameters>* mutable_parameters() { return &params_; }
  bool has_key() const { return has_key_; }
  const DpfKey& key() const { return key_; }
  DpfKey* mutable_key() { has_key_ = true; return &key_; }
  int32_t previous_hierarchy_level() const { return prev_; }
  void set_previous_hierarchy_level(int32_t v) { prev_ = v; }
  int partial_evaluations_size() const { return partials_.size(); }
  const PartialEvaluation& partial_evaluations(int i) const { return partials_[i]; }
  PartialEvaluation* add_partial_evaluations() { return partials_.Add(); }
  const RepeatedField<PartialEvaluation>& partial_evaluations() const { return partials_; }
  RepeatedField<PartialEvaluation>* mutable_partial_evaluations() { return &partials_; }
  void clear_partial_evaluations() { partials_.Clear(); }
  int32_t partial_evaluations_level() const { return partials_level_; }
  void set_partial_evaluations_level(int32_t v) { partials_level_ = v; }
  DPF_PROTO_MESSAGE_API(EvaluationContext)

 private:
  RepeatedField<DpfParameters> params_;
  bool has_key_ = false;
  DpfKey key_;
  int32_t prev_ = 0;
  RepeatedField<PartialEvaluation> partials_;
  int32_t partials_level_ = 0;
};

// Out-of-line accessors that need complete types.
inline const Value& Value_Tuple::elements(int i) const { return elements_[i]; }
inline Value* Value_Tuple::mutable_elements(int i) { return elements_.Mutable(i); }
inline Value* Value_Tuple::add_elements() { return elements_.Add(); }
inline const ValueType& ValueType_Tuple::elements(int i) const { return elements_[i]; }
inline ValueType* ValueType_Tuple::mutable_elements(int i) { return &const_cast<ValueType&>(elements_[i]); }
inline ValueType* ValueType_Tuple::add_elements() { return elements_.Add(); }
inline const Block& Value_Integer::value_uint128() const {
  static const Block kEmpty;
  return case_ == kValueUint128 ? u128_ : kEmpty;
}
inline const Value_Integer& Value::integer() const {
  static const Value_Integer kEmpty;
  return case_ == kInteger ? int_ : kEmpty;
}
inline const Value_Tuple& Value::tuple() const {
  static const Value_Tuple kEmpty;
  return case_ == kTuple ? tuple_ : kEmpty;
}
inline const Value_Integer& Value::int_mod_n() const {
  static const Value_Integer kEmpty;
  return case_ == kIntModN ? int_ : kEmpty;
}
inline const Value_Integer& Value::xor_wrapper() const {
  static const Value_Integer kEmpty;
  return case_ == kXorWrapper ? int_ : kEmpty;
}
inline const ValueType_Integer& ValueType::integer() const {
  static const ValueType_Integer kEmpty;
  return case_ == kInteger ? int_ : kEmpty;
}
inline const ValueType_Tuple& ValueType::tuple() const {
  static const ValueType_Tuple kEmpty;
  return case_ == kTuple ? tuple_ : kEmpty;
}
inline const ValueType_IntModN& ValueType::int_mod_n() const {
  static const ValueType_IntModN kEmpty;
  return case_ == kIntModN ? mod_ : kEmpty;
}
inline const ValueType_Integer& ValueType::xor_wrapper() const {
  static const ValueType_Integer kEmpty;
  return case_ == kXorWrapper ? int_ : kEmpty;
}

}  // namespace distributed_point_functions

#endif  // DPF_DISTRIBUTED_POINT_FUNCTION_PB_H_
