// The host worker pool behind the library's parallel loops
// (csrc/host/value_type_helpers.cc RunOnPool): a parallel loop
// nested inside a chunk -- on the submitting thread or on a worker -- runs
// inline and completes; an exception thrown by a chunk reaches the caller
// and leaves the pool usable; several threads submitting at once all finish;
// a forked child gets a working pool of its own.
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <functional>
#include <stdexcept>
#include <thread>
#include <vector>

namespace distributed_point_functions {
namespace dpf_internal {
void RunOnPool(int chunks, const std::function<void(int)>& fn);
}  // namespace dpf_internal
}  // namespace distributed_point_functions

using distributed_point_functions::dpf_internal::RunOnPool;

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);  \
      ++failures;                                                 \
    }                                                             \
  } while (0)

static int64_t NestedSum(int outer, int inner) {
  std::atomic<int64_t> sum{0};
  RunOnPool(outer, [&](int c) {
    RunOnPool(inner, [&](int d) { sum += c * 1000 + d; });
  });
  return sum.load();
}

int main() {
  // Nested loops (chunk 0 runs on the submitting thread).
  int64_t want = 0;
  for (int c = 0; c < 8; ++c)
    for (int d = 0; d < 5; ++d) want += c * 1000 + d;
  for (int rep = 0; rep < 50; ++rep) CHECK(NestedSum(8, 5) == want);

  // A throwing chunk: the first exception reaches the caller, the pool stays usable.
  for (int rep = 0; rep < 20; ++rep) {
    bool caught = false;
    try {
      RunOnPool(8, [&](int c) {
        if (c == 3) throw std::runtime_error("chunk 3");
      });
    } catch (const std::runtime_error&) {
      caught = true;
    }
    CHECK(caught);
    // ... and when the throwing chunk is nested.
    caught = false;
    try {
      RunOnPool(4, [&](int c) {
        RunOnPool(3, [&](int d) {
          if (c == 0 && d == 2) throw std::runtime_error("nested");
        });
      });
    } catch (const std::runtime_error&) {
      caught = true;
    }
    CHECK(caught);
    CHECK(NestedSum(8, 5) == want);
  }

  // Several submitting threads at once (the losers run on threads of their own).
  std::vector<std::thread> ts;
  std::atomic<int> ok{0};
  for (int t = 0; t < 6; ++t)
    ts.emplace_back([&] {
      for (int rep = 0; rep < 20; ++rep)
        if (NestedSum(6, 4) == [] {
              int64_t w = 0;
              for (int c = 0; c < 6; ++c)
                for (int d = 0; d < 4; ++d) w += c * 1000 + d;
              return w;
            }())
          ++ok;
    });
  for (auto& t : ts) t.join();
  CHECK(ok.load() == 6 * 20);

  // fork() while another thread keeps the pool busy: the child's pool works.
  std::atomic<bool> stop{false};
  std::thread busy([&] {
    while (!stop.load()) (void)NestedSum(8, 2);
  });
  const pid_t pid = fork();
  if (pid == 0) {
    const bool good = NestedSum(8, 5) == want;
    _exit(good ? 0 : 1);
  }
  int status = 0;
  CHECK(pid > 0 && waitpid(pid, &status, 0) == pid);
  CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  stop = true;
  busy.join();

  std::printf("%d failures\n", failures);
  return failures ? 1 : 0;
}
