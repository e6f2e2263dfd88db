// proto_validator.h -- validation of DpfParameters / DpfKey / EvaluationContext
// and the hierarchy-level <-> tree-level mapping (behaviour of the reference's
// dpf/internal/proto_validator.{h,cc}).
#ifndef DPF_INTERNAL_PROTO_VALIDATOR_H_
#define DPF_INTERNAL_PROTO_VALIDATOR_H_

#include <map>
#include <memory>
#include <vector>

#include "dpf/distributed_point_function.pb.h"
#include "dpf/span.h"
#include "dpf/status.h"

namespace distributed_point_functions {
namespace dpf_internal {

class ProtoValidator {
 public:
  // proto_validator.h:35-38
  static constexpr double kDefaultSecurityParameter = 40;
  static constexpr double kSecurityParameterEpsilon = 0.0001;

  static StatusOr<std::unique_ptr<ProtoValidator>> Create(Span<const DpfParameters> parameters);
  static Status ValidateParameters(Span<const DpfParameters> parameters);
  Status ValidateDpfKey(const DpfKey& key) const;
  Status ValidateEvaluationContext(const EvaluationContext& ctx) const;
  static Status ValidateValueType(const ValueType& value_type);
  static Status ValidateValue(const Value& value, const ValueType& type);
  Status ValidateValue(const Value& value, int i) const {
    return ValidateValue(value, parameters_[i].value_type());
  }

  ProtoValidator(const ProtoValidator&) = delete;
  ProtoValidator& operator=(const ProtoValidator&) = delete;

  Span<const DpfParameters> parameters() const { return MakeConstSpan(parameters_); }
  int tree_levels_needed() const { return tree_levels_needed_; }
  const std::map<int, int>& tree_to_hierarchy() const { return tree_to_hierarchy_; }
  const std::vector<int>& hierarchy_to_tree() const { return hierarchy_to_tree_; }

 private:
  ProtoValidator(std::vector<DpfParameters> parameters, int tree_levels_needed,
                 std::map<int, int> tree_to_hierarchy, std::vector<int> hierarchy_to_tree)
      : parameters_(std::move(parameters)),
        tree_levels_needed_(tree_levels_needed),
        tree_to_hierarchy_(std::move(tree_to_hierarchy)),
        hierarchy_to_tree_(std::move(hierarchy_to_tree)) {}

  std::vector<DpfParameters> parameters_;
  int tree_levels_needed_;
  std::map<int, int> tree_to_hierarchy_;
  std::vector<int> hierarchy_to_tree_;
};

}  // namespace dpf_internal
}  // namespace distributed_point_functions

#endif  // DPF_INTERNAL_PROTO_VALIDATOR_H_
