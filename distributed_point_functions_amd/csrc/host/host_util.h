// host_util.h -- helpers shared by the host C++ sources: PRG keys, uint128 <->
// dpf_block / proto Block conversion, C-ABI status mapping, the value-type
// descriptor handed to the kernels, and reusable device allocations.
#ifndef DPF_HOST_HOST_UTIL_H_
#define DPF_HOST_HOST_UTIL_H_

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "dpf/span.h"

#include "dpf/distributed_point_function.pb.h"
#include "dpf/internal/value_type_helpers.h"
#include "dpf/status.h"
#include "dpf/uint128.h"
#include "dpf_hip.h"

namespace distributed_point_functions {
namespace dpf_internal {

// PRG keys (distributed_point_function.cc:32-42): first half of SHA256 of the
// constant names.
constexpr uint128 kPrgKeyLeft = MakeUint128(0x5be037ccf6a03de5ULL, 0x935f08d0a5b6a2fdULL);
constexpr uint128 kPrgKeyRight = MakeUint128(0xef94b6aedebb026cULL, 0xe2ea1fe0f66f4d0bULL);
constexpr uint128 kPrgKeyValue = MakeUint128(0x05a5d1588c5423e3ULL, 0x46a31101b21d1c98ULL);

inline Status FromHip(int code) {
  if (code == 0) return OkStatus();
  return Status(static_cast<StatusCode>(code), dpf_hip_last_error());
}
#define HIP_RETURN_IF_ERROR(expr) DPF_RETURN_IF_ERROR(::distributed_point_functions::dpf_internal::FromHip(expr))

// Events marking how much of a device output produced in parts on one stream
// is complete: part j = [0, ends[j]) once events[j] has completed.
class PartEvents {
 public:
  PartEvents() = default;
  PartEvents(const PartEvents&) = delete;
  PartEvents& operator=(const PartEvents&) = delete;
  ~PartEvents() {
    for (void* e : events_) {
      (void)dpf_hip_event_sync(e);
      dpf_hip_event_destroy(e);
    }
  }
  Status Record(size_t end, void* stream) {
    void* e = nullptr;
    HIP_RETURN_IF_ERROR(dpf_hip_event_create(&e));
    events_.push_back(e);
    ends_.push_back(end);
    return FromHip(dpf_hip_event_record(e, stream));
  }
  int size() const { return static_cast<int>(events_.size()); }
  void* const* events() const { return events_.data(); }
  const size_t* ends() const { return ends_.data(); }

 private:
  std::vector<void*> events_;
  std::vector<size_t> ends_;
};

// Results of kOverlapGrowMin bytes up to below kOverlapGrowLimit that arrive
// through the staging buffers are value-initialised on a helper thread
// during the DMA (CopyToHostSink).  Measured: uint64/20 466 -> 364 us,
// uint128/20 845 -> 646 us, Tuple<uint32_t x5>/20 (20 MiB) 1.46 -> 1.03 ms
// (profiles/r15_ab.txt part 20).  From 32 MiB, glibc hands out fresh mmap
// pages, whose faults the helper would take alone and ahead of every copy,
// where chunk by chunk they overlap the next chunk's DMA (uint128/22
// 7.4 -> 9.7 ms grown whole); below 4 MiB a thread costs about what it
// saves.  DPF_OVERLAP_GROW=0 (read per call) grows them chunk by chunk as
// before (A/B and test hook).
constexpr size_t kOverlapGrowMin = size_t{4} << 20;
constexpr size_t kOverlapGrowLimit = size_t{32} << 20;
inline bool OverlapGrowOn() {
  const char* v = std::getenv("DPF_OVERLAP_GROW");
  return !(v && v[0] == '0');
}

// Copies `bytes` of device output into the storage `dst` a HostSink reserved,
// letting its grow() initialise each chunk right before that chunk's DMA
// (dpf_hip_memcpy_d2h_staged; with `parts`, each chunk's DMA waits only for
// the part that covers it, dpf_hip_memcpy_d2h_staged_after).  Returns a
// dpf_hip status code.
inline int CopyToHostSink(const HostSink& sink, void* dst, const void* src, size_t bytes,
                          void* stream, const PartEvents* parts = nullptr) {
  if (sink.chunk && (!dst || bytes < DPF_HIP_REGISTER_MIN_BYTES)) {
    auto consume = [](void* ctx, const void* chunk, size_t offset, size_t len) {
      (*static_cast<const HostSink*>(ctx)).chunk(static_cast<const uint8_t*>(chunk), offset, len);
    };
    if (sink.grow && bytes >= kOverlapGrowMin && bytes < kOverlapGrowLimit && OverlapGrowOn()) {
      // The result's one-thread value-initialisation (~60 GB/s) runs on a
      // helper thread while the first chunk's DMA is in flight; the chunks
      // are then copied (or unpacked) into the grown result in parallel.
      struct Ctx {
        const HostSink* sink;
        std::thread helper;
        bool joined = false;
        bool failed = false;
        void Join() {
          if (!joined) helper.join();
          joined = true;
        }
      } ctx{&sink, {}};
      try {
        ctx.helper = std::thread([&ctx, bytes] {
          try {
            ctx.sink->grow(bytes);
          } catch (...) {
            ctx.failed = true;
          }
        });
      } catch (...) {
        return dpf_hip_memcpy_d2h_chunked(src, bytes, sink.align, consume,
                                          const_cast<HostSink*>(&sink), stream);
      }
      auto consume_grown = [](void* c, const void* chunk, size_t offset, size_t len) {
        Ctx& x = *static_cast<Ctx*>(c);
        x.Join();
        if (x.failed) throw std::bad_alloc();
        x.sink->chunk(static_cast<const uint8_t*>(chunk), offset, len);
      };
      const int rc = dpf_hip_memcpy_d2h_chunked(src, bytes, sink.align, consume_grown, &ctx, stream);
      ctx.Join();
      return rc;
    }
    return dpf_hip_memcpy_d2h_chunked(src, bytes, sink.align, consume,
                                      const_cast<HostSink*>(&sink), stream);
  }
  if (!sink.grow) return dpf_hip_memcpy_d2h(dst, src, bytes, stream);
  auto before = [](void* ctx, size_t ready) {
    (*static_cast<const std::function<void(size_t)>*>(ctx))(ready);
  };
  if (parts && parts->size() > 0)
    return dpf_hip_memcpy_d2h_staged_after(
        dst, src, bytes, before, const_cast<std::function<void(size_t)>*>(&sink.grow),
        parts->size(), parts->events(), parts->ends(), stream);
  return dpf_hip_memcpy_d2h_staged(dst, src, bytes, before,
                                   const_cast<std::function<void(size_t)>*>(&sink.grow), stream);
}

// `bytes` of device memory into a fresh host vector.
inline int CopyToHostVector(std::vector<uint8_t>* out, const void* src, size_t bytes, void* stream) {
  const HostSink sink = VectorSink(out);
  return CopyToHostSink(sink, sink.reserve(bytes), src, bytes, stream);
}

inline dpf_block ToBlock(uint128 v) { return dpf_block{Uint128Low64(v), Uint128High64(v)}; }
inline uint128 FromBlock(const dpf_block& b) { return MakeUint128(b.high, b.low); }
inline uint128 FromProtoBlock(const Block& b) { return MakeUint128(b.high(), b.low()); }
inline void SetProtoBlock(uint128 v, Block* b) {
  b->set_high(Uint128High64(v));
  b->set_low(Uint128Low64(v));
}

inline dpf_aes_key AesKey(uint128 k) {
  dpf_aes_key r;
  std::memcpy(r.bytes, &k, 16);
  return r;
}

inline dpf_value_desc MakeDesc(const FlatValueType& f, int blocks_needed) {
  dpf_value_desc d;
  std::memset(&d, 0, sizeof(d));
  d.num_leaves = static_cast<int32_t>(f.leaves.size());
  d.direct = f.direct ? 1 : 0;
  d.elements_per_block = f.elements_per_block;
  d.blocks_needed = blocks_needed;
  for (size_t k = 0; k < f.leaves.size() && k < DPF_MAX_LEAVES; ++k) {
    d.kind[k] = f.leaves[k].kind;
    d.bits[k] = f.leaves[k].bits;
    d.mod_low[k] = Uint128Low64(f.leaves[k].modulus);
    d.mod_high[k] = Uint128High64(f.leaves[k].modulus);
  }
  return d;
}

struct U128Hash {
  size_t operator()(uint128 v) const {
    uint64_t x = Uint128Low64(v) * 0x9E3779B97F4A7C15ULL ^ Uint128High64(v);
    x ^= x >> 29;
    return static_cast<size_t>(x * 0xBF58476D1CE4E5B9ULL);
  }
};

// Host threads the library's parallel loops may use: DPF_HOST_THREADS when
// set (>= 1), else min(16, hardware threads) -- 16 is the GPU box's CPU share
// per GPU.
inline int HostThreads() {
  static const int n = [] {
    const char* e = std::getenv("DPF_HOST_THREADS");
    const int v = e ? std::atoi(e) : 0;
    if (v >= 1) return v;
    return static_cast<int>(std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency())));
  }();
  return n;
}

// Runs fn(c) for every c in [0, chunks) on the library's persistent host
// worker pool (HostThreads() - 1 workers, started on first use) with the
// calling thread taking part; returns when all chunks are done, rethrowing
// the first exception a chunk threw.  Spawning threads per call cost ~20 us
// each -- more than the work at mid sizes (the EvaluateAt point pass and
// unpack, r15).  Calls made from a pool worker run their chunks inline; a
// call that finds the pool busy with another thread's job starts threads of
// its own.
void RunOnPool(int chunks, const std::function<void(int)>& fn);

// fn(lo, hi) over [0, n) split across host threads (at most HostThreads())
// when n is large enough to pay for them; inline otherwise.
template <typename F>
void ParallelFor(int64_t n, F fn, int64_t min_per_thread = int64_t{1} << 15) {
  int threads = static_cast<int>(std::min<int64_t>(
      HostThreads(), n / std::max<int64_t>(min_per_thread, 1)));
  if (threads <= 1) {
    if (n > 0) fn(int64_t{0}, n);
    return;
  }
  RunOnPool(threads, [&](int t) { fn(n * t / threads, n * (t + 1) / threads); });
}

// Number of chunks ParallelChunks uses for n items.
inline int NumChunks(int64_t n, int64_t min_per_chunk = int64_t{1} << 15) {
  return static_cast<int>(std::max<int64_t>(
      1, std::min<int64_t>(HostThreads(), n / std::max<int64_t>(min_per_chunk, 1))));
}

// fn(chunk, lo, hi) for `chunks` contiguous chunks of [0, n), one thread each.
template <typename F>
void ParallelChunks(int64_t n, int chunks, F fn) {
  if (chunks <= 1) {
    fn(0, int64_t{0}, n);
    return;
  }
  RunOnPool(chunks, [&](int c) { fn(c, n * c / chunks, n * (c + 1) / chunks); });
}

// Unique tree indices (prefix >> bib) of `prefixes` in first-seen order and,
// per prefix, (position of its tree index, block index) -- EvaluateUntil's
// dedup (distributed_point_function.h:718-742).  Ascending prefixes (the
// hierarchical case) take a two-pass parallel scan; anything else a hash map.
// The output vectors are overwritten (their capacity is reused).
// `*ascending_out` (if given) tells whether the tree indices came out strictly
// ascending (ascending prefixes).
// `Pos` is the position type of prefix_map (int32_t halves its memory traffic
// where the caller bounds the tree indices below 2^31).
template <typename Pos>
void DedupTreeIndices(Span<const uint128> prefixes, int bib, std::vector<uint128>* tree_indices,
                      std::vector<std::pair<Pos, int>>* prefix_map, bool* ascending_out = nullptr) {
  const int64_t P = static_cast<int64_t>(prefixes.size());
  if (ascending_out) *ascending_out = false;
  if (P == 0) {
    tree_indices->clear();
    prefix_map->clear();
    return;
  }
  const uint128 bmask = (static_cast<uint128>(1) << bib) - 1;
  const int chunks = NumChunks(P);
  auto starts = [&](int64_t i) {
    return i == 0 || (prefixes[i] >> bib) != (prefixes[i - 1] >> bib);
  };
  // One pass checks the order and counts each chunk's tree-index starts (the
  // host side of a 1 M-prefix level is bound by memory traffic, config 5a).
  std::vector<char> chunk_ascending(chunks, 1);
  std::vector<int64_t> first(chunks + 1, 0);
  ParallelChunks(P, chunks, [&](int c, int64_t lo, int64_t hi) {
    int64_t k = lo == 0 ? 1 : 0;
    for (int64_t i = std::max<int64_t>(lo, 1); i < hi; ++i) {
      if (!(prefixes[i - 1] < prefixes[i])) {
        chunk_ascending[c] = 0;
        return;
      }
      k += starts(i);
    }
    first[c + 1] = k;
  });
  const bool ascending =
      std::all_of(chunk_ascending.begin(), chunk_ascending.end(), [](char a) { return a != 0; });
  if (ascending) {
    if (ascending_out) *ascending_out = true;
    // Equal tree indices are adjacent: scan the starts per chunk, place.
    for (int c = 0; c < chunks; ++c) first[c + 1] += first[c];
    // Every element is overwritten below: vectors kept from an earlier call
    // (the caller's scratch) only value-initialise what they grow by.
    tree_indices->resize(first[chunks]);
    prefix_map->resize(P);
    ParallelChunks(P, chunks, [&](int c, int64_t lo, int64_t hi) {
      int64_t pos = first[c] - 1;
      for (int64_t i = lo; i < hi; ++i) {
        if (starts(i)) (*tree_indices)[++pos] = prefixes[i] >> bib;
        (*prefix_map)[i] = {static_cast<Pos>(pos), static_cast<int>(prefixes[i] & bmask)};
      }
    });
    return;
  }
  std::unordered_map<uint128, int64_t, U128Hash> inverse;
  inverse.reserve(P * 2);
  tree_indices->clear();
  prefix_map->clear();
  tree_indices->reserve(P);
  prefix_map->reserve(P);
  for (int64_t i = 0; i < P; ++i) {
    const uint128 ti = prefixes[i] >> bib;
    auto [it, inserted] = inverse.try_emplace(ti, static_cast<int64_t>(tree_indices->size()));
    if (inserted) tree_indices->push_back(ti);
    prefix_map->emplace_back(static_cast<Pos>(it->second), static_cast<int>(prefixes[i] & bmask));
  }
}

// A growable device allocation (C-ABI allocator), reused across calls.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  ~DeviceBuffer() {
    if (p_) dpf_hip_free(p_);
  }
  Status Reserve(size_t bytes) {
    if (bytes <= cap_ && p_) return OkStatus();
    if (p_) dpf_hip_free(p_);
    p_ = nullptr;
    cap_ = 0;
    size_t want = std::max<size_t>(bytes, 256);
    HIP_RETURN_IF_ERROR(dpf_hip_alloc(&p_, want));
    cap_ = want;
    return OkStatus();
  }
  // Copies on `stream` (ordered after earlier work on it) and waits.
  template <typename T>
  Status Upload(const T* data, size_t count, void* stream = nullptr) {
    DPF_RETURN_IF_ERROR(Reserve(count * sizeof(T)));
    return FromHip(dpf_hip_memcpy_h2d(p_, data, count * sizeof(T), stream));
  }
  void* get() const { return p_; }
  size_t capacity() const { return cap_; }
  template <typename T>
  T* as() const { return static_cast<T*>(p_); }

 private:
  void* p_ = nullptr;
  size_t cap_ = 0;
};

// Small uploads go through one page-locked ring: the bytes are copied into
// it and the H2D copy is queued without waiting, so the kernel that consumes
// them follows on the same stream (a call used to pay one copy + stream
// synchronisation per argument array, ~18 us each).  The ring wraps only
// after every stream that copied from it has been synchronised.  Uploads
// larger than kMaxStaged take the synchronous pageable path.
class HostStaging {
 public:
  static constexpr size_t kMaxStaged = size_t{4} << 20;
  HostStaging() = default;
  HostStaging(const HostStaging&) = delete;
  HostStaging& operator=(const HostStaging&) = delete;
  ~HostStaging() {
    (void)Drain();
    for (void* e : free_events_) dpf_hip_event_destroy(e);
    if (p_) dpf_hip_host_free(p_);
  }
  Status Upload(DeviceBuffer& dst, const void* data, size_t bytes, void* stream) {
    DPF_RETURN_IF_ERROR(dst.Reserve(bytes));
    if (bytes == 0) return OkStatus();
    if (bytes > kMaxStaged) return FromHip(dpf_hip_memcpy_h2d(dst.get(), data, bytes, stream));
    if (used_ + bytes > cap_) {
      DPF_RETURN_IF_ERROR(Drain());
      used_ = 0;
      if (bytes > cap_) {
        if (p_) dpf_hip_host_free(p_);
        p_ = nullptr;
        cap_ = 0;
        const size_t want = std::max<size_t>(kMaxStaged, bytes);
        HIP_RETURN_IF_ERROR(dpf_hip_host_alloc(&p_, want));
        cap_ = want;
      }
    }
    char* src = static_cast<char*>(p_) + used_;
    std::memcpy(src, data, bytes);
    HIP_RETURN_IF_ERROR(dpf_hip_memcpy_h2d_async(dst.get(), src, bytes, stream));
    used_ += (bytes + 255) & ~size_t{255};
    // One event per stream since the last wrap, re-recorded after each copy.
    for (auto& [st, ev] : pending_)
      if (st == stream) return FromHip(dpf_hip_event_record(ev, stream));
    void* ev = nullptr;
    if (!free_events_.empty()) {
      ev = free_events_.back();
      free_events_.pop_back();
    } else {
      HIP_RETURN_IF_ERROR(dpf_hip_event_create(&ev));
    }
    pending_.emplace_back(stream, ev);
    return FromHip(dpf_hip_event_record(ev, stream));
  }

 private:
  Status Drain() {
    for (auto& [st, ev] : pending_) {
      HIP_RETURN_IF_ERROR(dpf_hip_event_sync(ev));
      free_events_.push_back(ev);
    }
    pending_.clear();
    return OkStatus();
  }
  void* p_ = nullptr;
  size_t cap_ = 0, used_ = 0;
  // (stream, event after its last copy) for copies from the ring since it wrapped.
  std::vector<std::pair<void*, void*>> pending_;
  std::vector<void*> free_events_;
};

// The argument arrays of ONE call packed into one image and copied with a
// single asynchronous H2D (a call's 6-8 separate copies cost ~5 us of API
// time each).  The image is built straight in page-locked memory (no second
// host pass over it before the DMA; callers may also fill an array in place:
// Reserve).  Usage: Reset(); [Prepare(total bytes)]; off = Add(data, n) or
// p = Reserve<T>(n, &off) per array; Commit(stream); then Ptr<T>(off) are the
// device addresses, valid until the next Reset().  Reset() waits for the
// previous call's stream, so neither the page-locked image nor the device
// arena is rewritten while a copy or kernel still reads it.  Images above
// kMaxPinned are built in pageable memory and copied synchronously.  Images
// of at most kZeroCopyMax (128 KiB) bytes are not copied at all: the kernels read them
// from the page-locked image itself (ROCm maps page-locked host memory into
// the device's address space), which saves a small call the ~5 us latency of
// one DMA (profiles/r13_latency_microbench.txt); DPF_UPLOAD_ZERO_COPY=0
// (read per call) copies them too (A/B and test hook).
class PackedUploads {
 public:
  PackedUploads() = default;
  PackedUploads(const PackedUploads&) = delete;
  PackedUploads& operator=(const PackedUploads&) = delete;
  ~PackedUploads() {
    if (pending_) (void)dpf_hip_event_sync(event_);
    if (event_) dpf_hip_event_destroy(event_);
    if (pinned_) dpf_hip_host_free(pinned_);
  }
  // Waits for the previous call's copy and kernel (an event recorded on its
  // stream after the launch, MarkUsed) before the buffers are rewritten.
  Status Reset() {
    if (pending_) {
      HIP_RETURN_IF_ERROR(dpf_hip_event_sync(event_));
    } else if (unmarked_) {
      // A zero-copy image whose caller returned before MarkUsed (an error
      // after Commit): whatever it launched may still read the image.
      HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(commit_stream_));
    }
    pending_ = false;
    unmarked_ = false;
    zero_copy_ = false;
    size_ = 0;
    pageable_ = false;
    return OkStatus();
  }
  // Room for `bytes` of arrays (each array 256-byte aligned): pointers from
  // Reserve stay valid until Commit only when the image never has to grow.
  void Prepare(size_t bytes) { Grow(bytes); }
  // Records that the work queued on `stream` so far reads the arena.
  Status MarkUsed(void* stream) {
    if (!event_) HIP_RETURN_IF_ERROR(dpf_hip_event_create(&event_));
    HIP_RETURN_IF_ERROR(dpf_hip_event_record(event_, stream));
    pending_ = true;
    unmarked_ = false;
    return OkStatus();
  }
  // Space for `count` elements of T in the image, to be filled by the caller
  // (valid until the image grows: Prepare first).
  template <typename T>
  T* Reserve(size_t count, size_t* off) {
    *off = (size_ + 255) & ~size_t{255};
    const size_t end = *off + std::max<size_t>(count * sizeof(T), 1);
    Grow(end);
    size_ = end;
    return reinterpret_cast<T*>(base() + *off);
  }
  template <typename T>
  size_t Add(const T* data, size_t count) {
    size_t off;
    T* p = Reserve<T>(count, &off);
    if (count) std::memcpy(p, data, count * sizeof(T));
    return off;
  }
  Status Commit(void* stream) {
    if (size_ == 0) return OkStatus();
    if (pageable_) {  // large batches: a synchronous copy from pageable memory
      DPF_RETURN_IF_ERROR(arena_.Reserve(size_));
      return FromHip(dpf_hip_memcpy_h2d(arena_.get(), image_.get(), size_, stream));
    }
    if (size_ <= kZeroCopyMax && ZeroCopyOn()) {
      zero_copy_ = true;
      unmarked_ = true;
      commit_stream_ = stream;
      return OkStatus();
    }
    DPF_RETURN_IF_ERROR(arena_.Reserve(cap_));
    HIP_RETURN_IF_ERROR(dpf_hip_memcpy_h2d_async(arena_.get(), pinned_, size_, stream));
    return MarkUsed(stream);
  }
  template <typename T>
  T* Ptr(size_t off) const {
    return reinterpret_cast<T*>((zero_copy_ ? static_cast<char*>(pinned_)
                                            : static_cast<char*>(arena_.get())) + off);
  }
  // True when this call's kernels read (and write) the host image itself.
  bool zero_copy() const { return zero_copy_; }

 private:
  static constexpr size_t kMaxPinned = size_t{64} << 20;
  static constexpr size_t kZeroCopyMax = size_t{128} << 10;
  static bool ZeroCopyOn() {
    const char* v = std::getenv("DPF_UPLOAD_ZERO_COPY");
    return !(v && v[0] == '0');
  }
  char* base() { return pageable_ ? image_.get() : static_cast<char*>(pinned_); }
  // Pageable image of at least `end` bytes holding [0, size_) of the current one
  // (uninitialised beyond: no value-initialisation pass over a large image).
  void GrowPageable(size_t end, const char* from) {
    if (image_ && image_cap_ >= end) {
      if (from != image_.get() && size_) std::memcpy(image_.get(), from, size_);
      return;
    }
    std::unique_ptr<char[]> ni(new char[end]);
    if (size_) std::memcpy(ni.get(), from, size_);
    image_ = std::move(ni);
    image_cap_ = end;
  }
  // Makes [0, end) of the image addressable, keeping [0, size_).
  void Grow(size_t end) {
    if (pageable_) {
      if (end > image_cap_) GrowPageable(std::max(end, image_cap_ + image_cap_ / 2), image_.get());
      return;
    }
    if (end <= cap_) return;
    void* np = nullptr;
    // Grow by half again, never past kMaxPinned (a long-lived
    // object must not keep ~1.5x the cap page-locked).
    const size_t want =
        std::max(end, std::min(std::max<size_t>(cap_ + cap_ / 2, size_t{1} << 20), kMaxPinned));
    if (end > kMaxPinned || dpf_hip_host_alloc(&np, want) != 0) {
      // Too large to keep page-locked (or no page-locked memory): pageable.
      GrowPageable(end, static_cast<const char*>(pinned_));
      pageable_ = true;
      return;
    }
    if (size_) std::memcpy(np, pinned_, size_);
    if (pinned_) dpf_hip_host_free(pinned_);
    pinned_ = np;
    cap_ = want;
  }
  std::unique_ptr<char[]> image_;  // pageable image (pageable_)
  size_t image_cap_ = 0;
  size_t size_ = 0;
  bool pageable_ = false;
  void* pinned_ = nullptr;
  size_t cap_ = 0;
  DeviceBuffer arena_;
  bool pending_ = false;
  bool zero_copy_ = false;   // this call's kernels read pinned_ itself
  bool unmarked_ = false;    // zero-copy Commit not yet followed by MarkUsed
  void* commit_stream_ = nullptr;
  void* event_ = nullptr;
};

// Orders reuse of a device buffer across calls that may come on different
// streams: Mark(stream) records an event after the last kernel that touches
// the buffer; Acquire(buf, bytes, stream) makes the next call's work wait for
// it -- on the device (hipStreamWaitEvent) when the stream differs, not at
// all on the same stream (stream order), and on the host only when the
// buffer must be reallocated (freeing memory a kernel may still use).
class StreamFence {
 public:
  StreamFence() = default;
  StreamFence(const StreamFence&) = delete;
  StreamFence& operator=(const StreamFence&) = delete;
  ~StreamFence() {
    if (pending_) (void)dpf_hip_event_sync(event_);
    if (event_) dpf_hip_event_destroy(event_);
  }
  Status Acquire(DeviceBuffer& buf, size_t bytes, void* stream) {
    if (pending_) {
      if (bytes > buf.capacity() || !buf.get()) {
        HIP_RETURN_IF_ERROR(dpf_hip_event_sync(event_));
        pending_ = false;
      } else if (stream != last_stream_) {
        HIP_RETURN_IF_ERROR(dpf_hip_stream_wait_event(stream, event_));
      }
    }
    return buf.Reserve(bytes);
  }
  Status Mark(void* stream) {
    if (!event_) HIP_RETURN_IF_ERROR(dpf_hip_event_create(&event_));
    HIP_RETURN_IF_ERROR(dpf_hip_event_record(event_, stream));
    pending_ = true;
    last_stream_ = stream;
    return OkStatus();
  }

 private:
  bool pending_ = false;
  void* event_ = nullptr;
  void* last_stream_ = nullptr;
};

// Page-locked memory for the result of a small call (<= 1 MiB): the kernel
// writes it over PCIe and the host reads it after a stream sync -- no D2H
// DMA and its ~5 us of latency (profiles/r13_latency_microbench.txt).  One
// 1 MiB buffer per DistributedPointFunction / DistributedComparisonFunction
// object, allocated at its first small call and freed with the object.
// DPF_OUTPUT_ZERO_COPY=0 (read per call) turns it off (A/B and test hook).
class PinnedOut {
 public:
  PinnedOut() = default;
  PinnedOut(const PinnedOut&) = delete;
  PinnedOut& operator=(const PinnedOut&) = delete;
  ~PinnedOut() {
    if (p_) dpf_hip_host_free(p_);
  }
  // Page-locked room for `bytes`, or nullptr (too large, off, or no memory).
  void* Get(size_t bytes) {
    const char* v = std::getenv("DPF_OUTPUT_ZERO_COPY");
    if (bytes == 0 || bytes > kMax || (v && v[0] == '0')) return nullptr;
    if (!p_ && dpf_hip_host_alloc(&p_, kMax) != 0) p_ = nullptr;
    return p_;
  }

 private:
  static constexpr size_t kMax = size_t{1} << 20;
  void* p_ = nullptr;
};

// Hands `bytes` of a result the kernels wrote to page-locked memory `p` (on
// `stream`) to a HostSink; a sink that throws (no memory for the result)
// is reported as an internal error, as the chunked D2H path does.
inline Status ConsumePinnedOut(const HostSink& sink, const void* p, size_t bytes, void* stream) {
  HIP_RETURN_IF_ERROR(dpf_hip_stream_sync(stream));
  try {
    void* dst = sink.reserve(bytes);
    if (sink.chunk) {
      sink.chunk(static_cast<const uint8_t*>(p), 0, bytes);
      return OkStatus();
    }
    if (sink.grow) sink.grow(bytes);
    std::memcpy(dst, p, bytes);
  } catch (const std::exception& e) {
    return InternalError(std::string("copying a small result to host memory failed: ") + e.what());
  }
  return OkStatus();
}

// The device buffers and staging of one DistributedPointFunction (or
// DistributedComparisonFunction).  The reference's const evaluation methods
// may be called from several threads at once; `mu` makes every call that
// uses these buffers take them in turn (recursive: a call's helpers lock too).
class DeviceScratch {
 public:
  std::recursive_mutex mu;
  PackedUploads packed;
  PackedUploads packed_pe;   // ComputePartialEvaluations' walk (its seeds feed the expansion)
  // EvaluateShardToDevice alternates between `packed` and this image, so a
  // call waits (PackedUploads::Reset) for the launch two calls back, not for
  // the one still running: back-to-back shard calls keep the GPU busy while
  // the host builds the next call's image.
  PackedUploads packed_alt;
  bool shard_alt = false;
  // EvaluateUntil's prefix dedup, kept across calls so a call of the same
  // size value-initialises nothing.
  std::vector<uint128> tree_indices;
  std::vector<std::pair<int64_t, int>> prefix_map;
  DeviceBuffer out, gathered, offsets, party, workspace;
  StreamFence workspace_fence;  // the sum kernels' 192-bit accumulators
  HostStaging staging;
  PinnedOut small_out;           // results of small calls, written by the kernels
  template <typename T>
  Status Upload(DeviceBuffer& dst, const T* data, size_t count, void* stream = nullptr) {
    return staging.Upload(dst, data, count * sizeof(T), stream);
  }
};

}  // namespace dpf_internal
}  // namespace distributed_point_functions

#endif  // DPF_HOST_HOST_UTIL_H_
