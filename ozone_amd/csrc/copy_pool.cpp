#include "copy_pool.hpp"

#include "numa.hpp"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

namespace ozec {
namespace {

constexpr size_t kPiece = 256 << 10;

// Streaming copy: every destination line is written whole with non-temporal stores, so the copy costs one read of
// the source and one write of the destination in DRAM -- a cached store first reads the line it writes (read for
// ownership), 3 DRAM transfers per byte instead of 2.  The staging copies feed DMA (the destination is read by the
// GPU's copy engine, not the CPU) or fill a caller's output buffer, so nothing is gained by leaving the destination
// in cache.  glibc switches to streaming stores only above several MiB, beyond the 256 KiB pieces copied here.
// The trailing sfence orders the streaming stores before the completion the copy signals (the DMA is queued after).
__attribute__((target("avx2"))) void copy_stream_avx2(void *dst, const void *src, size_t n) {
  char *d = static_cast<char *>(dst);
  const char *s = static_cast<const char *>(src);
  const size_t head = std::min(n, static_cast<size_t>((32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31));
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  for (; n >= 128; n -= 128, d += 128, s += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d), a);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i *>(d + 96), e);
  }
  std::memcpy(d, s, n);
  _mm_sfence();
}

// -1 auto (= 1 where AVX2 exists), 0 memcpy, 1 streaming stores both ways, 2 streaming stores into staging buffers
// only (the copies whose destination only the DMA engine reads).  Same-process A/Bs on two boxes
// (profiles/r03/ab/copy*_*.log): 16 callers 6 % / 27 % faster with streaming stores, the pageable stripe queue 11 % /
// 25 %, one caller 3.7 % slower on one box and 3.6 % faster on the other.  `shared` (a copy that shares DRAM with
// other transfers) is kept for A/Bs of a policy that streams only then (mode 3).
std::atomic<int> g_stream_mode{-1};

bool use_stream(CopyDir dir, bool shared) {
  int m = g_stream_mode.load(std::memory_order_relaxed);
  if (m < 0) m = __builtin_cpu_supports("avx2") ? 1 : 0;
  if (m == 3) return shared && __builtin_cpu_supports("avx2");
  return m == 1 || (m == 2 && dir == CopyDir::kToStaging);
}

void copy_bytes(void *dst, const void *src, size_t n, bool stream) {
  if (stream && n >= 4096) copy_stream_avx2(dst, src, n);
  else std::memcpy(dst, src, n);
}

struct Job {
  std::vector<CopyTask> pieces;
  bool stream = false;
  std::atomic<size_t> next{0};
  std::atomic<size_t> done{0};
  std::mutex mu;
  std::condition_variable cv;

  // copy pieces until none are left; returns after contributing
  void work() {
    for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
      copy_bytes(pieces[i].dst, pieces[i].src, pieces[i].n, stream);
      if (done.fetch_add(1) + 1 == pieces.size()) {
        std::lock_guard<std::mutex> lk(mu);
        cv.notify_all();
      }
    }
  }
};

// copy_spin (ozec_set_tuning "copy_spin_us"): how long a pool worker, and a caller waiting for its job's last pieces,
// poll before sleeping on a condition variable (0: sleep at once)
std::atomic<int64_t> g_spin_ns{0};

template <class Pred>
void spin_until(Pred done) {
  const int64_t ns = g_spin_ns.load(std::memory_order_relaxed);
  if (ns <= 0) return;
  const auto end = std::chrono::steady_clock::now() + std::chrono::nanoseconds(ns);
  while (!done()) {
    for (int i = 0; i < 64; ++i) _mm_pause();
    if (std::chrono::steady_clock::now() >= end) return;
  }
}

// One pool per host NUMA node: a GPU's staging buffers live on its node (numa.hpp), and the copies into and out of
// them run on that node's CPUs -- a process driving GPUs on both sockets (devices.hpp) keeps every staging copy local.
int g_default_threads = -1;  // -1: min(8, hardware threads / 2) - 1, or OZEC_COPY_THREADS

class Pool {
 public:
  explicit Pool(int node) : node_(node) { start_workers(default_threads()); }
  ~Pool() { stop_workers(); }

  static int default_threads() {
    if (g_default_threads >= 0) return g_default_threads;
    int n = static_cast<int>(std::min(8u, std::max(1u, std::thread::hardware_concurrency() / 2)) - 1);
    if (const char *e = std::getenv("OZEC_COPY_THREADS")) n = std::max(0, std::atoi(e));
    return n;
  }

  void resize(int n) {
    std::lock_guard<std::mutex> lk(resize_mu_);
    const int keep = nthreads_;
    stop_workers();
    start_workers(n < 0 ? keep : n);
  }

  int size() const { return nthreads_; }

  void run(const std::shared_ptr<Job> &job) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back(job);
      epoch_.fetch_add(1);
    }
    cv_.notify_all();
    job->work();
    spin_until([&] { return job->done.load() == job->pieces.size(); });
    std::unique_lock<std::mutex> lk(job->mu);
    job->cv.wait(lk, [&] { return job->done.load() == job->pieces.size(); });
  }

 private:
  void start_workers(int n) {
    stop_ = false;
    nthreads_ = n;
    for (int i = 0; i < n; ++i)
      workers_.emplace_back([this, node = node_] {
        (void)bind_thread_to_node(node);
        loop();
      });
  }

  void stop_workers() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
    workers_.clear();
    nthreads_ = 0;
  }

  void loop() {
    uint64_t seen = epoch_.load();
    for (;;) {
      // a worker that just finished keeps polling for copy_spin before it sleeps: the staging copies of a pipelined
      // call come every few tens of microseconds, and a futex wake-up costs about as much as a 256 KiB piece
      spin_until([&] { return epoch_.load() != seen || stop_.load(); });
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        seen = epoch_.load();
        if (stop_) return;
        job = jobs_.front();
        if (job->next.load() >= job->pieces.size()) {  // fully claimed: retire it
          jobs_.pop_front();
          continue;
        }
      }
      job->work();
    }
  }

  std::mutex resize_mu_, mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Job>> jobs_;
  std::vector<std::thread> workers_;
  std::atomic<uint64_t> epoch_{0};  // jobs queued so far (the spinning workers' signal)
  std::atomic<bool> stop_{false};
  int nthreads_ = 0;
  int node_ = -1;
};

std::mutex g_pools_mu;
std::map<int, std::unique_ptr<Pool>> g_pools;  // by NUMA node (-1: unknown / not NUMA); never destroyed before exit

Pool &pool_for(int node) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  auto &p = g_pools[node];
  if (!p) p.reset(new Pool(node));
  return *p;
}

}  // namespace

void set_copy_threads(int n) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  g_default_threads = std::max(0, n);
  for (auto &kv : g_pools) kv.second->resize(g_default_threads);
}

void set_copy_spin_us(int64_t us) { g_spin_ns.store(std::max<int64_t>(0, us) * 1000); }

int64_t copy_spin_us() { return g_spin_ns.load() / 1000; }

bool set_copy_stream(int mode) {
  if (mode < -1 || mode > 3) return false;
  g_stream_mode.store(mode);
  return true;
}

void parallel_copy(const std::vector<CopyTask> &tasks, CopyDir dir, bool shared, int node) {
  size_t total = 0;
  for (const CopyTask &t : tasks) total += t.n;
  const bool stream = use_stream(dir, shared);
  Pool &pool = pool_for(node);
  if (pool.size() == 0 || total < 2 * kPiece) {
    for (const CopyTask &t : tasks) copy_bytes(t.dst, t.src, t.n, stream);
    return;
  }
  auto job = std::make_shared<Job>();
  job->stream = stream;
  for (const CopyTask &t : tasks)
    for (size_t off = 0; off < t.n; off += kPiece)
      job->pieces.push_back({static_cast<char *>(t.dst) + off, static_cast<const char *>(t.src) + off,
                             std::min(kPiece, t.n - off)});
  pool.run(job);
}

}  // namespace ozec
