#include "copy_pool.hpp"

#include "numa.hpp"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

namespace ozec {
namespace {

constexpr size_t kPiece = 256 << 10;

struct Job {
  std::vector<CopyTask> pieces;
  std::atomic<size_t> next{0};
  std::atomic<size_t> done{0};
  std::mutex mu;
  std::condition_variable cv;

  // copy pieces until none are left; returns after contributing
  void work() {
    for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
      std::memcpy(pieces[i].dst, pieces[i].src, pieces[i].n);
      if (done.fetch_add(1) + 1 == pieces.size()) {
        std::lock_guard<std::mutex> lk(mu);
        cv.notify_all();
      }
    }
  }
};

class Pool {
 public:
  static Pool &get() {
    static Pool p;
    return p;
  }

  void resize(int n) {
    std::lock_guard<std::mutex> lk(resize_mu_);
    const int keep = nthreads_;
    stop_workers();
    start_workers(n < 0 ? keep : n);
  }

  // restart the workers on the CPUs of `node` (the first GPU this process uses: its staging buffers live there)
  void set_node(int node) {
    std::lock_guard<std::mutex> lk(resize_mu_);
    if (node == node_) return;
    const int n = nthreads_;
    stop_workers();
    node_ = node;
    start_workers(n);
  }

  int size() const { return nthreads_; }

  void run(const std::shared_ptr<Job> &job) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back(job);
    }
    cv_.notify_all();
    job->work();
    std::unique_lock<std::mutex> lk(job->mu);
    job->cv.wait(lk, [&] { return job->done.load() == job->pieces.size(); });
  }

 private:
  Pool() {
    int n = static_cast<int>(std::min(8u, std::max(1u, std::thread::hardware_concurrency() / 2)) - 1);
    if (const char *e = std::getenv("OZEC_COPY_THREADS")) n = std::max(0, std::atoi(e));
    start_workers(n);
  }
  ~Pool() { stop_workers(); }

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
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
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
  bool stop_ = false;
  int nthreads_ = 0;
  int node_ = -1;
};

}  // namespace

void set_copy_threads(int n) { Pool::get().resize(std::max(0, n)); }

void set_copy_node(int node) { Pool::get().set_node(node); }

void parallel_copy(const std::vector<CopyTask> &tasks) {
  size_t total = 0;
  for (const CopyTask &t : tasks) total += t.n;
  Pool &pool = Pool::get();
  if (pool.size() == 0 || total < 2 * kPiece) {
    for (const CopyTask &t : tasks) std::memcpy(t.dst, t.src, t.n);
    return;
  }
  auto job = std::make_shared<Job>();
  for (const CopyTask &t : tasks)
    for (size_t off = 0; off < t.n; off += kPiece)
      job->pieces.push_back({static_cast<char *>(t.dst) + off, static_cast<const char *>(t.src) + off,
                             std::min(kPiece, t.n - off)});
  pool.run(job);
}

}  // namespace ozec
