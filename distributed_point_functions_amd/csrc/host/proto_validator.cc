// proto_validator.cc -- restates dpf/internal/proto_validator.cc (file:line
// references below are to that file).
#include "dpf/internal/proto_validator.h"

#include <cmath>
#include <string>

#include "dpf/internal/value_type_helpers.h"

namespace distributed_point_functions {
namespace dpf_internal {
namespace {

double DefaultSecurityParameter(const DpfParameters& p) {
  return ProtoValidator::kDefaultSecurityParameter + p.log_domain_size();  // :27-30
}

bool AlmostEqual(double a, double b) {
  return std::abs(a - b) <= ProtoValidator::kSecurityParameterEpsilon;  // :32-34
}

StatusOr<bool> ParametersAreEqual(const DpfParameters& lhs, const DpfParameters& rhs) {
  // :36-56
  if (lhs.log_domain_size() != rhs.log_domain_size()) return false;
  if (!(AlmostEqual(lhs.security_parameter(), rhs.security_parameter()) ||
        (lhs.security_parameter() == 0 &&
         AlmostEqual(rhs.security_parameter(), DefaultSecurityParameter(rhs))) ||
        (rhs.security_parameter() == 0 &&
         AlmostEqual(lhs.security_parameter(), DefaultSecurityParameter(lhs))))) {
    return false;
  }
  return ValueTypesAreEqual(lhs.value_type(), rhs.value_type());
}

Status ValidateIntegerType(const ValueType::Integer& type) {
  // :58-71
  int bitsize = type.bitsize();
  if (bitsize < 1) return InvalidArgumentError("`bitsize` must be positive");
  if (bitsize > 128) return InvalidArgumentError("`bitsize` must be less than or equal to 128");
  if ((bitsize & (bitsize - 1)) != 0) return InvalidArgumentError("`bitsize` must be a power of 2");
  return OkStatus();
}

Status ValidateIntegerValue(const Value::Integer& value, const ValueType::Integer& type) {
  // :73-84
  if (type.bitsize() < 128) {
    DPF_ASSIGN_OR_RETURN(uint128 v, ValueIntegerToUint128(value));
    if (v >= (static_cast<uint128>(1) << type.bitsize())) {
      return InvalidArgumentError("Value (= " + Uint128ToString(v) +
                                  ") too large for ValueType with bitsize = " +
                                  std::to_string(type.bitsize()));
    }
  }
  return OkStatus();
}

}  // namespace

StatusOr<std::unique_ptr<ProtoValidator>> ProtoValidator::Create(
    Span<const DpfParameters> parameters_in) {
  // :97-142
  DPF_RETURN_IF_ERROR(ValidateParameters(parameters_in));
  std::vector<DpfParameters> parameters(parameters_in.begin(), parameters_in.end());
  for (DpfParameters& p : parameters)
    if (p.security_parameter() == 0) p.set_security_parameter(DefaultSecurityParameter(p));
  std::map<int, int> tree_to_hierarchy;
  std::vector<int> hierarchy_to_tree(parameters.size());
  int tree_levels_needed = 0;
  for (int i = 0; i < static_cast<int>(parameters.size()); ++i) {
    DPF_ASSIGN_OR_RETURN(int bits_needed,
                         BitsNeeded(parameters[i].value_type(), parameters[i].security_parameter()));
    int log_bits_needed = static_cast<int>(std::ceil(std::log2(bits_needed)));
    int tree_level = std::max(tree_levels_needed,
                              parameters[i].log_domain_size() - 7 + std::min(log_bits_needed, 7));
    tree_to_hierarchy[tree_level] = i;
    hierarchy_to_tree[i] = tree_level;
    tree_levels_needed = std::max(tree_levels_needed, tree_level + 1);
  }
  return std::unique_ptr<ProtoValidator>(new ProtoValidator(
      std::move(parameters), tree_levels_needed, std::move(tree_to_hierarchy),
      std::move(hierarchy_to_tree)));
}

Status ProtoValidator::ValidateParameters(Span<const DpfParameters> parameters) {
  // :144-187
  if (parameters.empty()) return InvalidArgumentError("`parameters` must not be empty");
  int previous_log_domain_size = 0;
  for (int i = 0; i < static_cast<int>(parameters.size()); ++i) {
    int log_domain_size = parameters[i].log_domain_size();
    if (log_domain_size < 0) return InvalidArgumentError("`log_domain_size` must be non-negative");
    if (log_domain_size > 128) return InvalidArgumentError("`log_domain_size` must be <= 128");
    if (i > 0 && log_domain_size <= previous_log_domain_size)
      return InvalidArgumentError(
          "`log_domain_size` fields must be in ascending order in `parameters`");
    previous_log_domain_size = log_domain_size;
    if (parameters[i].has_value_type()) {
      DPF_RETURN_IF_ERROR(ValidateValueType(parameters[i].value_type()));
    } else {
      return InvalidArgumentError("`value_type` is required");
    }
    if (std::isnan(parameters[i].security_parameter()))
      return InvalidArgumentError("`security_parameter` must not be NaN");
    if (parameters[i].security_parameter() < 0 || parameters[i].security_parameter() > 128)
      return InvalidArgumentError("`security_parameter` must be in [0, 128]");
  }
  return OkStatus();
}

Status ProtoValidator::ValidateDpfKey(const DpfKey& key) const {
  // :189-220
  if (!key.has_seed()) return InvalidArgumentError("key.seed must be present");
  if (key.last_level_value_correction().empty())
    return InvalidArgumentError("key.last_level_value_correction must be present");
  if (key.correction_words_size() != tree_levels_needed_ - 1)
    return InvalidArgumentError("Malformed DpfKey: expected " +
                                std::to_string(tree_levels_needed_ - 1) +
                                " correction words, but got " +
                                std::to_string(key.correction_words_size()));
  for (int i = 0; i < static_cast<int>(hierarchy_to_tree_.size()); ++i) {
    if (hierarchy_to_tree_[i] == tree_levels_needed_ - 1) continue;
    if (key.correction_words(hierarchy_to_tree_[i]).value_correction().empty())
      return InvalidArgumentError("Malformed DpfKey: expected correction_words[" +
                                  std::to_string(hierarchy_to_tree_[i]) +
                                  "] to contain the value correction of hierarchy level " +
                                  std::to_string(i));
  }
  return OkStatus();
}

Status ProtoValidator::ValidateEvaluationContext(const EvaluationContext& ctx) const {
  // :222-251
  if (ctx.parameters_size() != static_cast<int>(parameters_.size()))
    return InvalidArgumentError("Number of parameters in `ctx` doesn't match");
  for (int i = 0; i < ctx.parameters_size(); ++i) {
    DPF_ASSIGN_OR_RETURN(bool eq, ParametersAreEqual(parameters_[i], ctx.parameters(i)));
    if (!eq) return InvalidArgumentError("Parameter " + std::to_string(i) + " in `ctx` doesn't match");
  }
  if (!ctx.has_key()) return InvalidArgumentError("ctx.key must be present");
  DPF_RETURN_IF_ERROR(ValidateDpfKey(ctx.key()));
  if (ctx.previous_hierarchy_level() >= ctx.parameters_size() - 1)
    return InvalidArgumentError("This context has already been fully evaluated");
  if (!ctx.partial_evaluations().empty() &&
      ctx.partial_evaluations_level() > ctx.previous_hierarchy_level())
    return InvalidArgumentError(
        "ctx.partial_evaluations_level must be less than or equal to "
        "ctx.previous_hierarchy_level");
  return OkStatus();
}

Status ProtoValidator::ValidateValueType(const ValueType& value_type) {
  // :253-271
  switch (value_type.type_case()) {
    case ValueType::kInteger:
      return ValidateIntegerType(value_type.integer());
    case ValueType::kTuple:
      for (const ValueType& el : value_type.tuple().elements())
        DPF_RETURN_IF_ERROR(ValidateValueType(el));
      return OkStatus();
    case ValueType::kIntModN:
      DPF_RETURN_IF_ERROR(ValidateIntegerType(value_type.int_mod_n().base_integer()));
      return ValidateIntegerValue(value_type.int_mod_n().modulus(),
                                  value_type.int_mod_n().base_integer());
    case ValueType::kXorWrapper:
      return ValidateIntegerType(value_type.xor_wrapper());
    default:
      return InvalidArgumentError("ValidateValueType: Unsupported ValueType:\n" +
                                  value_type.DebugString());
  }
}

Status ProtoValidator::ValidateValue(const Value& value, const ValueType& type) {
  // :273-317
  switch (type.type_case()) {
    case ValueType::kInteger:
      if (value.value_case() != Value::kInteger) return InvalidArgumentError("Expected integer value");
      return ValidateIntegerValue(value.integer(), type.integer());
    case ValueType::kTuple:
      if (value.value_case() != Value::kTuple) return InvalidArgumentError("Expected tuple value");
      if (value.tuple().elements_size() != type.tuple().elements_size())
        return InvalidArgumentError("Expected tuple value of size " +
                                    std::to_string(type.tuple().elements_size()) +
                                    " but got size " + std::to_string(value.tuple().elements_size()));
      for (int i = 0; i < type.tuple().elements_size(); ++i)
        DPF_RETURN_IF_ERROR(ValidateValue(value.tuple().elements(i), type.tuple().elements(i)));
      return OkStatus();
    case ValueType::kIntModN: {
      DPF_RETURN_IF_ERROR(ValidateIntegerValue(value.int_mod_n(), type.int_mod_n().base_integer()));
      DPF_ASSIGN_OR_RETURN(uint128 v, ValueIntegerToUint128(value.int_mod_n()));
      DPF_ASSIGN_OR_RETURN(uint128 m, ValueIntegerToUint128(type.int_mod_n().modulus()));
      if (v >= m)
        return InvalidArgumentError("Value (= " + Uint128ToString(v) +
                                    ") is too large for modulus (= " + Uint128ToString(m) + ")");
      return OkStatus();
    }
    case ValueType::kXorWrapper:
      if (value.value_case() != Value::kXorWrapper)
        return InvalidArgumentError("Expected XorWrapper value");
      return ValidateIntegerValue(value.xor_wrapper(), type.xor_wrapper());
    default:
      return InvalidArgumentError("ValidateValue: Unsupported ValueType:\n" + type.DebugString());
  }
}

}  // namespace dpf_internal
}  // namespace distributed_point_functions
