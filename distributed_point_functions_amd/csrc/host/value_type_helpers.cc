// value_type_helpers.cc -- runtime value-type semantics for the host API.
// Behaviour restated from the reference (file:line references are to
// dpf/internal/value_type_helpers.{h,cc} and dpf/int_mod_n.{h,cc} unless noted).
#include "dpf/internal/value_type_helpers.h"

#include <pthread.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <thread>

#include <sys/mman.h>

#include <cmath>
#include <string>

#include "host_util.h"

namespace distributed_point_functions {
namespace dpf_internal {
namespace {

uint128 Mask(int bits) { return bits >= 128 ? Uint128Max() : ((static_cast<uint128>(1) << bits) - 1); }

uint128 LoadLE(const uint8_t* p, int n) {
  uint128 v = 0;
  for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

Status FlattenInto(const ValueType& t, FlatValueType* f) {
  switch (t.type_case()) {
    case ValueType::kInteger:
      f->leaves.push_back({kLeafInt, t.integer().bitsize(), 0});
      return OkStatus();
    case ValueType::kXorWrapper:
      f->leaves.push_back({kLeafXor, t.xor_wrapper().bitsize(), 0});
      return OkStatus();
    case ValueType::kIntModN: {
      DPF_ASSIGN_OR_RETURN(uint128 m, ValueIntegerToUint128(t.int_mod_n().modulus()));
      f->leaves.push_back({kLeafIntModN, t.int_mod_n().base_integer().bitsize(), m});
      f->direct = false;
      return OkStatus();
    }
    case ValueType::kTuple:
      for (const ValueType& e : t.tuple().elements()) DPF_RETURN_IF_ERROR(FlattenInto(e, f));
      return OkStatus();
    default:
      return InvalidArgumentError("Flatten: Unsupported ValueType:\n" + t.DebugString());
  }
}

// Uint128To<T> (h:151-162): only the low 64 bits are range-checked.
StatusOr<uint128> CheckIntegerRange(uint128 v, int bits) {
  if (bits < 128) {
    uint64_t max = bits >= 64 ? ~uint64_t{0} : ((uint64_t{1} << bits) - 1);
    if (Uint128Low64(v) > max) {
      return InvalidArgumentError("Value (= " + std::to_string(Uint128Low64(v)) +
                                  ") too large for the given type T (size " +
                                  std::to_string(bits / 8) + ")");
    }
    return v & Mask(bits);
  }
  return v;
}

Status ValueToLeavesInto(const ValueType& type, const Value& value, std::vector<uint128>* out) {
  switch (type.type_case()) {
    case ValueType::kInteger: {
      // h:171-183
      if (value.value_case() != Value::kInteger)
        return InvalidArgumentError("The given Value is not an integer");
      DPF_ASSIGN_OR_RETURN(uint128 v, ValueIntegerToUint128(value.integer()));
      DPF_ASSIGN_OR_RETURN(uint128 r, CheckIntegerRange(v, type.integer().bitsize()));
      out->push_back(r);
      return OkStatus();
    }
    case ValueType::kIntModN: {
      // h:254-269
      if (value.value_case() != Value::kIntModN)
        return InvalidArgumentError("The given Value is not an IntModN");
      DPF_ASSIGN_OR_RETURN(uint128 v, ValueIntegerToUint128(value.int_mod_n()));
      DPF_ASSIGN_OR_RETURN(uint128 m, ValueIntegerToUint128(type.int_mod_n().modulus()));
      if (v >= m)
        return InvalidArgumentError("The given value (= " + Uint128ToString(v) +
                                    ") is larger than kModulus (= " + Uint128ToString(m) + ")");
      out->push_back(v);
      return OkStatus();
    }
    case ValueType::kXorWrapper: {
      // h:460-471 (no value-case check: a missing field reads as an unset Integer)
      DPF_ASSIGN_OR_RETURN(uint128 v, ValueIntegerToUint128(value.xor_wrapper()));
      DPF_ASSIGN_OR_RETURN(uint128 r, CheckIntegerRange(v, type.xor_wrapper().bitsize()));
      out->push_back(r);
      return OkStatus();
    }
    case ValueType::kTuple: {
      // h:346-382
      if (value.value_case() != Value::kTuple)
        return InvalidArgumentError("The given Value is not a tuple");
      if (value.tuple().elements_size() != type.tuple().elements_size())
        return InvalidArgumentError(
            "The tuple in the given Value has the wrong number of elements");
      for (int i = 0; i < type.tuple().elements_size(); ++i)
        DPF_RETURN_IF_ERROR(ValueToLeavesInto(type.tuple().elements(i), value.tuple().elements(i), out));
      return OkStatus();
    }
    default:
      return InvalidArgumentError("Unsupported ValueType");
  }
}

}  // namespace

StatusOr<FlatValueType> Flatten(const ValueType& value_type) {
  FlatValueType f;
  DPF_RETURN_IF_ERROR(FlattenInto(value_type, &f));
  for (const LeafSpec& l : f.leaves) {
    f.total_bits += l.bits;
    f.packed_size += (l.bits + 7) / 8;
  }
  f.elements_per_block =
      (f.direct && f.total_bits > 0 && f.total_bits <= 128) ? 128 / f.total_bits : 1;
  return f;
}

StatusOr<bool> ValueTypesAreEqual(const ValueType& lhs, const ValueType& rhs) {
  // value_type_helpers.cc:22-58
  if (lhs.type_case() == ValueType::TYPE_NOT_SET || rhs.type_case() == ValueType::TYPE_NOT_SET)
    return InvalidArgumentError("Both arguments must be valid ValueTypes");
  if (lhs.type_case() == ValueType::kInteger && rhs.type_case() == ValueType::kInteger)
    return lhs.integer().bitsize() == rhs.integer().bitsize();
  if (lhs.type_case() == ValueType::kTuple && rhs.type_case() == ValueType::kTuple &&
      lhs.tuple().elements_size() == rhs.tuple().elements_size()) {
    bool result = true;
    for (int i = 0; i < lhs.tuple().elements_size(); ++i) {
      DPF_ASSIGN_OR_RETURN(bool e, ValueTypesAreEqual(lhs.tuple().elements(i), rhs.tuple().elements(i)));
      result &= e;
    }
    return result;
  }
  if (lhs.type_case() == ValueType::kIntModN && rhs.type_case() == ValueType::kIntModN) {
    DPF_ASSIGN_OR_RETURN(uint128 lm, ValueIntegerToUint128(lhs.int_mod_n().modulus()));
    DPF_ASSIGN_OR_RETURN(uint128 rm, ValueIntegerToUint128(rhs.int_mod_n().modulus()));
    return lhs.int_mod_n().base_integer().bitsize() == rhs.int_mod_n().base_integer().bitsize() &&
           lm == rm;
  }
  if (lhs.type_case() == ValueType::kXorWrapper && rhs.type_case() == ValueType::kXorWrapper)
    return lhs.xor_wrapper().bitsize() == rhs.xor_wrapper().bitsize();
  return false;
}

double IntModNBase::GetSecurityLevel(int num_samples, uint128 modulus) {
  // int_mod_n.cc:21-26
  return 128 + 3 -
         (std::log2(static_cast<double>(modulus)) + std::log2(static_cast<double>(num_samples)) +
          std::log2(static_cast<double>(num_samples + 1)));
}

Status IntModNBase::CheckParameters(int num_samples, int base_integer_bitsize, uint128 modulus,
                                    double security_parameter) {
  // int_mod_n.cc:28-61
  if (num_samples <= 0) return InvalidArgumentError("num_samples must be positive");
  if (base_integer_bitsize <= 0) return InvalidArgumentError("base_integer_bitsize must be positive");
  if (base_integer_bitsize > 128)
    return InvalidArgumentError("base_integer_bitsize must be at most 128");
  if (base_integer_bitsize < 128 && (static_cast<uint128>(1) << base_integer_bitsize) < modulus)
    return InvalidArgumentError("kModulus " + Uint128ToString(modulus) +
                                " out of range for base_integer_bitsize = " +
                                std::to_string(base_integer_bitsize));
  const double sigma = GetSecurityLevel(num_samples, modulus);
  if (security_parameter > sigma) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%f", sigma);
    return InvalidArgumentError("For num_samples = " + std::to_string(num_samples) +
                                " and kModulus = " + Uint128ToString(modulus) +
                                " this approach can only provide " + buf +
                                " bits of statistical security. You can try calling this function "
                                "several times with smaller values of num_samples.");
  }
  return OkStatus();
}

StatusOr<int> IntModNBase::GetNumBytesRequired(int num_samples, int base_integer_bitsize,
                                               uint128 modulus, double security_parameter) {
  // int_mod_n.cc:63-76
  DPF_RETURN_IF_ERROR(
      CheckParameters(num_samples, base_integer_bitsize, modulus, security_parameter));
  return 16 + ((base_integer_bitsize + 7) / 8) * (num_samples - 1);
}

StatusOr<int> BitsNeeded(const ValueType& value_type, double security_parameter) {
  // value_type_helpers.cc:60-130, including the recursion into the *first*
  // num_other elements of a tuple (:94-103).
  switch (value_type.type_case()) {
    case ValueType::kInteger:
      return value_type.integer().bitsize();
    case ValueType::kTuple: {
      int num_mod = 0, num_other = 0;
      const ValueType* mod = nullptr;
      for (const ValueType& el : value_type.tuple().elements()) {
        if (el.type_case() == ValueType::kIntModN) {
          if (!mod) {
            mod = &el;
          } else {
            DPF_ASSIGN_OR_RETURN(bool eq, ValueTypesAreEqual(el, *mod));
            if (!eq)
              return UnimplementedError("All elements of type IntModN in a tuple must be the same");
          }
          ++num_mod;
        } else {
          ++num_other;
        }
      }
      int bits_other = 0, bits_mod = 0;
      for (int i = 0; i < num_other; ++i) {
        double per = security_parameter + std::log2(static_cast<double>(num_other));
        DPF_ASSIGN_OR_RETURN(int b, BitsNeeded(value_type.tuple().elements(i), per));
        bits_other += b;
      }
      if (num_mod > 0) {
        DPF_ASSIGN_OR_RETURN(uint128 m, ValueIntegerToUint128(mod->int_mod_n().modulus()));
        DPF_ASSIGN_OR_RETURN(int bytes, IntModNNumBytesRequired(
                                            num_mod, mod->int_mod_n().base_integer().bitsize(), m,
                                            security_parameter));
        bits_mod = bytes * 8;
      }
      return bits_mod + bits_other;
    }
    case ValueType::kIntModN: {
      DPF_ASSIGN_OR_RETURN(uint128 m, ValueIntegerToUint128(value_type.int_mod_n().modulus()));
      DPF_ASSIGN_OR_RETURN(int bytes, IntModNNumBytesRequired(
                                          1, value_type.int_mod_n().base_integer().bitsize(), m,
                                          security_parameter));
      return 8 * bytes;
    }
    case ValueType::kXorWrapper:
      return value_type.xor_wrapper().bitsize();
    default:
      return InvalidArgumentError("BitsNeeded: Unsupported ValueType:\n" + value_type.DebugString());
  }
}

Value::Integer Uint128ToValueInteger(uint128 in) {
  // value_type_helpers.cc:134-144
  Value::Integer r;
  if (Uint128High64(in) == 0) {
    r.set_value_uint64(Uint128Low64(in));
  } else {
    r.mutable_value_uint128()->set_high(Uint128High64(in));
    r.mutable_value_uint128()->set_low(Uint128Low64(in));
  }
  return r;
}

StatusOr<uint128> ValueIntegerToUint128(const Value::Integer& in) {
  // value_type_helpers.cc:146-155
  if (in.value_case() == Value::Integer::kValueUint128)
    return MakeUint128(in.value_uint128().high(), in.value_uint128().low());
  if (in.value_case() == Value::Integer::kValueUint64) return static_cast<uint128>(in.value_uint64());
  return InvalidArgumentError("Unknown value case for the given integer Value");
}

std::string SerializeValueTypeDeterministically(const ValueType& value_type) {
  return value_type.SerializeAsString();
}

StatusOr<std::vector<uint128>> ValueToLeaves(const ValueType& type, const Value& value) {
  std::vector<uint128> out;
  DPF_RETURN_IF_ERROR(ValueToLeavesInto(type, value, &out));
  return out;
}

Value LeavesToValue(const ValueType& type, const uint128* leaves, int* pos) {
  Value r;
  switch (type.type_case()) {
    case ValueType::kInteger: *r.mutable_integer() = Uint128ToValueInteger(leaves[(*pos)++]); break;
    case ValueType::kIntModN: *r.mutable_int_mod_n() = Uint128ToValueInteger(leaves[(*pos)++]); break;
    case ValueType::kXorWrapper:
      *r.mutable_xor_wrapper() = Uint128ToValueInteger(leaves[(*pos)++]);
      break;
    case ValueType::kTuple: {
      Value::Tuple* t = r.mutable_tuple();
      for (const ValueType& e : type.tuple().elements()) *t->add_elements() = LeavesToValue(e, leaves, pos);
      break;
    }
    default: break;
  }
  return r;
}

StatusOr<std::vector<uint128>> ValuesToLeafArray(const ValueType& type, const FlatValueType& flat,
                                                 const RepeatedField<Value>& values) {
  // ValuesToArray (h:544-563)
  if (values.size() != flat.elements_per_block)
    return InvalidArgumentError("values.size() (= " + std::to_string(values.size()) +
                                ") does not match ElementsPerBlock<T>() (= " +
                                std::to_string(flat.elements_per_block) + ")");
  std::vector<uint128> out;
  out.reserve(flat.elements_per_block * flat.leaves.size());
  for (const Value& v : values) DPF_RETURN_IF_ERROR(ValueToLeavesInto(type, v, &out));
  return out;
}

void ConvertBytesToLeaves(const FlatValueType& flat, const uint8_t* bytes, uint128* out) {
  const int nl = static_cast<int>(flat.leaves.size());
  if (flat.direct) {
    // DirectlyFromBytes for integers (h:199-211) and tuples (h:415-428).
    const int esz = (flat.total_bits + 7) / 8;
    for (int e = 0; e < flat.elements_per_block; ++e) {
      int off = e * esz;
      for (int k = 0; k < nl; ++k) {
        int lb = flat.leaves[k].bits / 8;
        out[e * nl + k] = LoadLE(bytes + off, lb);
        off += lb;
      }
    }
    return;
  }
  // FromBytes via SampleAndUpdateBytes (h:213-234, 286-311, 430-443, 531-538).
  uint128 block = LoadLE(bytes, 16);
  const uint8_t* rem = bytes + 16;
  for (int k = 0; k < nl; ++k) {
    const LeafSpec& s = flat.leaves[k];
    const bool update = k + 1 < nl;
    const int lb = s.bits / 8;
    if (s.kind == kLeafIntModN) {
      uint128 q = block / s.modulus;
      out[k] = block - q * s.modulus;
      if (update) {
        block = lb < 16 ? (q << (8 * lb)) : 0;
        block |= LoadLE(rem, lb);
        rem += lb;
      }
    } else {
      out[k] = block & Mask(s.bits);
      if (update) {
        if (lb < 16) block &= ~Mask(s.bits); else block = 0;
        block |= LoadLE(rem, lb);
        rem += lb;
      }
    }
  }
}

uint128 LeafAdd(const LeafSpec& s, uint128 a, uint128 b) {
  switch (s.kind) {
    case kLeafXor: return a ^ b;
    case kLeafIntModN: return LeafSub(s, a, s.modulus - b);  // AddBaseInteger
    default: return (a + b) & Mask(s.bits);
  }
}
uint128 LeafSub(const LeafSpec& s, uint128 a, uint128 b) {
  switch (s.kind) {
    case kLeafXor: return a ^ b;
    case kLeafIntModN: return a >= b ? a - b : s.modulus - b + a;  // SubtractBaseInteger
    default: return (a - b) & Mask(s.bits);
  }
}
uint128 LeafNeg(const LeafSpec& s, uint128 a) {
  switch (s.kind) {
    case kLeafXor: return a;
    case kLeafIntModN: return LeafSub(s, 0, a);
    default: return (0 - a) & Mask(s.bits);
  }
}

void PackLeaves(const FlatValueType& flat, const uint128* leaves, uint8_t* out) {
  for (size_t k = 0; k < flat.leaves.size(); ++k) {
    int lb = flat.leaves[k].bits / 8;
    uint128 v = leaves[k];
    for (int i = 0; i < lb; ++i) { out[i] = static_cast<uint8_t>(v); v >>= 8; }
    out += lb;
  }
}

void UnpackLeaves(const FlatValueType& flat, const uint8_t* in, uint128* leaves) {
  for (size_t k = 0; k < flat.leaves.size(); ++k) {
    int lb = flat.leaves[k].bits / 8;
    leaves[k] = LoadLE(in, lb);
    in += lb;
  }
}

void AdviseHugePages(void* p, size_t bytes) {
  constexpr uintptr_t kHuge = uintptr_t{2} << 20;
  if (!p || bytes < (size_t{4} << 20)) return;
  const uintptr_t lo = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t hi = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
  if (hi > lo) (void)madvise(reinterpret_cast<void*>(lo), hi - lo, MADV_HUGEPAGE);
}

const void* ZeroPages(size_t* bytes) {
  constexpr size_t kSpan = size_t{64} << 20;
  // Never written: every page reads as the kernel's shared zero page, so a
  // memmove out of it reads from cache.  Null (and resize()) if mmap fails.
  static const void* const zeros = [] {
    void* p = mmap(nullptr, kSpan, PROT_READ, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    return p == MAP_FAILED ? static_cast<const void*>(nullptr) : static_cast<const void*>(p);
  }();
  *bytes = zeros ? kSpan : 0;
  return zeros;
}

void PrefaultPages(void* p, size_t bytes) {
  if (!p || bytes < (size_t{64} << 20)) return;
  constexpr size_t kPage = 4096;
  volatile char* base = static_cast<char*>(p);
  const int64_t pages = static_cast<int64_t>(bytes / kPage);
  ParallelChunks(pages, NumChunks(pages, 4096), [base](int, int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) base[i * kPage] = 0;
  });
}

namespace {
// The persistent worker pool behind RunOnPool (host_util.h).  Workers and
// the caller spin briefly on the job generation / completion counters before
// sleeping, so back-to-back parallel loops (the ~10-100 us phases of one
// EvaluateAt call) do not pay a futex wake-up per worker.
class WorkerPool {
 public:
  explicit WorkerPool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { Loop(); });
  }
  int workers() const { return static_cast<int>(threads_.size()); }
  // False if another thread's job is running.  The submitting thread is
  // marked (in_job) while it runs chunks, so a nested parallel loop inside a
  // chunk runs inline instead of try_lock-ing submit_, which it already owns
  // (undefined behaviour for a std::mutex).
  bool TryRun(int chunks, const std::function<void(int)>& fn) {
    std::unique_lock<std::mutex> submit(submit_, std::try_to_lock);
    if (!submit.owns_lock()) return false;
    struct JobMark {
      JobMark() { in_job = true; }
      ~JobMark() { in_job = false; }
    } mark;
    {
      std::lock_guard<std::mutex> lock(mu_);
      fn_ = &fn;
      chunks_ = chunks;
      next_.store(0);
      error_ = nullptr;
      active_.store(workers());
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    Work(chunks, fn);
    SpinUntil([this] { return active_.load(std::memory_order_acquire) == 0; });
    if (active_.load(std::memory_order_acquire) != 0) {
      std::unique_lock<std::mutex> lock(mu_);
      done_cv_.wait(lock, [this] { return active_.load() == 0; });
    }
    std::lock_guard<std::mutex> lock(mu_);
    fn_ = nullptr;
    if (error_) std::rethrow_exception(error_);
    return true;
  }
  static thread_local bool in_worker;
  static thread_local bool in_job;   // this thread submitted the running job

 private:
  // Polls `done` for up to ~50 us (yielding the CPU between polls: a pause
  // loop can cost a VM exit per iteration on virtualised hosts), then gives up.
  template <typename P>
  static void SpinUntil(P done) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(50);
    while (!done()) {
      for (int i = 0; i < 64 && !done(); ++i) {
      }
      if (done() || std::chrono::steady_clock::now() > until) return;
      std::this_thread::yield();
    }
  }
  void Work(int chunks, const std::function<void(int)>& fn) {
    for (int c = next_.fetch_add(1); c < chunks; c = next_.fetch_add(1)) {
      try {
        fn(c);
      } catch (...) {
        std::lock_guard<std::mutex> lock(mu_);
        if (!error_) error_ = std::current_exception();
      }
    }
  }
  void Loop() {
    in_worker = true;
    uint64_t seen = 0;
    for (;;) {
      SpinUntil([&] { return gen_.load(std::memory_order_acquire) != seen; });
      const std::function<void(int)>* fn;
      int chunks;
      {
        std::unique_lock<std::mutex> lock(mu_);
        cv_.wait(lock, [&] { return gen_.load() != seen; });
        seen = gen_.load();
        fn = fn_;
        chunks = chunks_;
      }
      Work(chunks, *fn);
      if (active_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> lock(mu_);
        done_cv_.notify_one();
      }
    }
  }
  std::mutex submit_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int chunks_ = 0;
  std::atomic<int> next_{0};
  std::atomic<int> active_{0};
  std::atomic<uint64_t> gen_{0};
  std::exception_ptr error_;
  std::vector<std::thread> threads_;
};
thread_local bool WorkerPool::in_worker = false;
thread_local bool WorkerPool::in_job = false;

// Never destroyed (its threads wait for work until the process exits); a
// forked child starts a pool of its own (the parent's threads do not exist
// there).  fork() takes g_pool_mu first (prepare handler), so the child never
// inherits it held by a thread that does not exist there; the child releases
// it and forgets the parent's pool, whose mutexes may be held by such threads.
std::atomic<WorkerPool*> g_pool{nullptr};
std::mutex g_pool_mu;
WorkerPool* Pool() {
  WorkerPool* p = g_pool.load();
  if (p) return p;
  static bool atfork = [] {
    pthread_atfork([] { g_pool_mu.lock(); }, [] { g_pool_mu.unlock(); },
                   [] {
                     g_pool_mu.unlock();
                     g_pool.store(nullptr);
                   });
    return true;
  }();
  (void)atfork;
  std::lock_guard<std::mutex> lock(g_pool_mu);
  if (!g_pool.load()) g_pool.store(new WorkerPool(std::max(HostThreads() - 1, 1)));
  return g_pool.load();
}
}  // namespace

void RunOnPool(int chunks, const std::function<void(int)>& fn) {
  if (chunks <= 1 || WorkerPool::in_worker || WorkerPool::in_job) {
    for (int c = 0; c < chunks; ++c) fn(c);
    return;
  }
  if (Pool()->TryRun(chunks, fn)) return;
  // The pool is busy with another thread's job: threads of this call's own.
  std::vector<std::thread> pool;
  std::exception_ptr error;
  std::mutex mu;
  auto run = [&](int c) {
    try {
      fn(c);
    } catch (...) {
      std::lock_guard<std::mutex> lock(mu);
      if (!error) error = std::current_exception();
    }
  };
  pool.reserve(chunks - 1);
  for (int c = 1; c < chunks; ++c) pool.emplace_back(run, c);
  run(0);
  for (auto& th : pool) th.join();
  if (error) std::rethrow_exception(error);
}

void ParallelRanges(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn) {
  ParallelChunks(n, NumChunks(n, grain), [&fn](int, int64_t lo, int64_t hi) { fn(lo, hi); });
}

}  // namespace dpf_internal

const char* StatusCodeToString(StatusCode code) {
  switch (code) {
    case StatusCode::kOk: return "OK";
    case StatusCode::kCancelled: return "CANCELLED";
    case StatusCode::kUnknown: return "UNKNOWN";
    case StatusCode::kInvalidArgument: return "INVALID_ARGUMENT";
    case StatusCode::kDeadlineExceeded: return "DEADLINE_EXCEEDED";
    case StatusCode::kNotFound: return "NOT_FOUND";
    case StatusCode::kAlreadyExists: return "ALREADY_EXISTS";
    case StatusCode::kPermissionDenied: return "PERMISSION_DENIED";
    case StatusCode::kResourceExhausted: return "RESOURCE_EXHAUSTED";
    case StatusCode::kFailedPrecondition: return "FAILED_PRECONDITION";
    case StatusCode::kAborted: return "ABORTED";
    case StatusCode::kOutOfRange: return "OUT_OF_RANGE";
    case StatusCode::kUnimplemented: return "UNIMPLEMENTED";
    case StatusCode::kInternal: return "INTERNAL";
    case StatusCode::kUnavailable: return "UNAVAILABLE";
    case StatusCode::kDataLoss: return "DATA_LOSS";
    case StatusCode::kUnauthenticated: return "UNAUTHENTICATED";
  }
  return "UNKNOWN";
}

}  // namespace distributed_point_functions
