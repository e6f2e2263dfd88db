// distributed_comparison_function.pb.h -- hand-written proto3 messages of
// dcf/distributed_comparison_function.proto (DcfParameters, DcfKey), wire
// compatible with the generated classes (field 1 = the wrapped DPF message).
#ifndef DCF_DISTRIBUTED_COMPARISON_FUNCTION_PB_H_
#define DCF_DISTRIBUTED_COMPARISON_FUNCTION_PB_H_

#include "dpf/distributed_point_function.pb.h"

namespace distributed_point_functions {

class DcfParameters {
 public:
  bool has_parameters() const { return has_params_; }
  const DpfParameters& parameters() const { return params_; }
  DpfParameters* mutable_parameters() { has_params_ = true; return &params_; }
  DPF_PROTO_MESSAGE_API(DcfParameters)

 private:
  bool has_params_ = false;
  DpfParameters params_;
};

class DcfKey {
 public:
  bool has_key() const { return has_key_; }
  const DpfKey& key() const { return key_; }
  DpfKey* mutable_key() { has_key_ = true; return &key_; }
  DPF_PROTO_MESSAGE_API(DcfKey)

 private:
  bool has_key_ = false;
  DpfKey key_;
};

}  // namespace distributed_point_functions

#endif  // DCF_DISTRIBUTED_COMPARISON_FUNCTION_PB_H_
