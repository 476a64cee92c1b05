// fs_plan -- the native round driver.
//
// One call enqueues the launches of one federated round of FedAvg / FedProx (and the
// local-training / aggregation / evaluation phases of FedAMW), replacing the per-round
// Python work of the reference's round loop (/root/reference/functions/tools.py:337-352,
// 364-379, 427-462):
//   TRAIN      fs_local_train over every client (train_loop, tools.py:340-343), losses
//              written straight into the [R][N] history
//   AGGREGATE  fs_aggregate: W_g = sum_j p_j W_j (tools.py:345-350)
//   EVAL       fs_eval of W_g on the test set into the [R][2] history (tools.py:351)
// The DataLoader shuffles of a round (tools.py:179, one RandomSampler permutation per
// client and epoch) are replayed bit-exactly (MT19937 + forward Fisher-Yates) into one of
// two slots on the plan's own side stream, so round t+1's shuffles are produced while
// round t trains:
//   shuffle_device = 1  fs_randperm_device (one wave per pass) after an async upload of
//                       the seeds from pinned memory -- a few hundred waves beside the
//                       local-training grid, no host work;
//   shuffle_device = 0  a persistent pool of host threads (as fs_randperm_batch) driven by
//                       a coordinator thread, then one async upload of the permutations.
// Events order the slots: a slot is rewritten only after the local training that
// consumed its previous contents, and a local training waits for its slot.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <deque>
#include <thread>
#include <vector>

#include <chrono>
#include <cstdio>

#include "common.h"
#include "finalize.h"
#include "mt_replay.h"

namespace fs {

// Persistent worker pool: run(n, fn) calls fn(i) for i in [0, n) on all workers + the caller.
class Pool {
 public:
  explicit Pool(int nthreads) {
    for (int t = 1; t < nthreads; ++t) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(int64_t n, const std::function<void(int64_t)>& fn) {
    if (th_.empty() || n <= 1) {
      for (int64_t i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      busy_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const int64_t i = next_.fetch_add(1);
      if (i >= n_) return;
      (*fn_)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      std::lock_guard<std::mutex> lk(m_);
      if (--busy_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  int busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace fs

struct fs_plan {
  fs_plan_desc d;
  std::vector<int64_t> n, off;         // per pass (j*E + e): rows, offset into the shuffle buffer
  int64_t perm_len = 0;                // E * rows
  int32_t* h_perm[2] = {nullptr, nullptr};   // pinned (host replay)
  int32_t* d_perm[2] = {nullptr, nullptr};
  // device replay: a ring of SEED_SLOTS pinned seed buffers, each freed by its own event, so the
  // host never waits on the shuffle of the previous round before enqueuing the next (with two
  // slots that wait held the host ~330 us per round at config 2 and left the GPU idle between
  // rounds -- r02s2t)
  static constexpr int SEED_SLOTS = 4;
  int64_t* h_seed[SEED_SLOTS] = {};             // pinned, coherent
  int64_t* d_seed[SEED_SLOTS] = {};
  int64_t* h_seed_dev[SEED_SLOTS] = {};         // device view of h_seed (zero-copy seeds)
  hipEvent_t seed_read[SEED_SLOTS] = {};
  bool seed_pending[SEED_SLOTS] = {};
  bool seed_copy = false;                         // FS_SEED_COPY=1: upload the seeds (hipMemcpyAsync)
  int64_t* d_pass = nullptr;                 // [2][P]: rows, offset of every pass (device replay)
  int64_t max_n = 0;
  int64_t max_client_steps = 0;       // E * ceil(max_j n_j / B)
  int fuse_E = 0;                     // evaluation blocks a TRAIN launch can carry (0: none)
  int eval_pending = -1;              // round whose evaluation rides on the next TRAIN launch
  int fin_pending = -1;               // round whose fused evaluation awaits its finaliser (it rides
                                      // on the next AGGREGATE launch, fs_plan_round)
  hipStream_t copy = nullptr;
  hipEvent_t uploaded[2] = {nullptr, nullptr};
  hipEvent_t consumed[2] = {nullptr, nullptr};
  bool up_pending[2] = {false, false};
  bool cons_recorded[2] = {false, false};
  int slot_round[2] = {-1, -1};       // round whose shuffles slot s holds (set by the coordinator)
  // chunked device replay (fs_plan_set_shuffle_chunk, K > 1): slot s holds the shuffles of
  // the K rounds of chunk c (rounds cK .. cK+K-1), generated by ONE launch; the local
  // training waits for the slot once per chunk and records its release once per chunk, so
  // consecutive rounds of a chunk run back to back with no cross-stream wait between them
  int chunk = 1;
  int64_t* d_pass_chunk = nullptr;    // [2][K*P]: rows, offset of every pass of a chunk
  int slot_chunk[2] = {-1, -1};       // chunk whose shuffles slot s holds (launched)
  int slot_nrounds[2] = {0, 0};       // rounds of that chunk generated
  int slot_waited[2] = {-1, -1};      // chunk the compute stream last waited for in slot s
  int fill_chunk = -1, fill_rounds = 0;   // chunk whose seeds are being collected, rounds so far
  int job_status = FS_OK;
  std::string job_error;
  fs::Pool* pool = nullptr;
  // coordinator: shuffle jobs (round, seeds) in order
  std::thread coord;
  std::mutex m;
  std::condition_variable cv, done;
  std::deque<std::pair<int, std::vector<int64_t>>> jobs;
  bool stop = false;
};

using namespace fs;

static int hip_fail(const char* what, hipError_t e) {
  return fail(FS_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define FS_HIP(call, what)                          \
  do {                                              \
    hipError_t e_ = (call);                         \
    if (e_ != hipSuccess) return hip_fail(what, e_); \
  } while (0)

extern "C" int64_t fs_plan_desc_size(void) { return (int64_t)sizeof(fs_plan_desc); }

static int run_shuffle_job(fs_plan* p, const int64_t* h_seeds, int t);

static void coordinator(fs_plan* p) {
  for (;;) {
    std::pair<int, std::vector<int64_t>> job;
    {
      std::unique_lock<std::mutex> lk(p->m);
      p->cv.wait(lk, [p] { return p->stop || !p->jobs.empty(); });
      if (p->jobs.empty()) return;
      job = std::move(p->jobs.front());
    }
    const int rc = run_shuffle_job(p, job.second.data(), job.first);
    std::lock_guard<std::mutex> lk(p->m);
    p->jobs.pop_front();
    if (rc != FS_OK && p->job_status == FS_OK) {
      p->job_status = rc;
      p->job_error = fs_last_error();
    }
    p->done.notify_all();
  }
}

extern "C" int fs_plan_destroy(fs_plan* p) {
  if (!p) return FS_OK;
  if (p->coord.joinable()) {
    {
      std::lock_guard<std::mutex> lk(p->m);
      p->stop = true;
    }
    p->cv.notify_all();
    p->coord.join();
  }
  if (p->copy) (void)hipStreamSynchronize(p->copy);
  for (int s = 0; s < 2; ++s) {
    if (p->h_perm[s]) (void)hipHostFree(p->h_perm[s]);
    if (p->d_perm[s]) (void)hipFree(p->d_perm[s]);
    if (p->uploaded[s]) (void)hipEventDestroy(p->uploaded[s]);
    if (p->consumed[s]) (void)hipEventDestroy(p->consumed[s]);
  }
  for (int s = 0; s < fs_plan::SEED_SLOTS; ++s) {
    if (p->h_seed[s]) (void)hipHostFree(p->h_seed[s]);
    if (p->d_seed[s]) (void)hipFree(p->d_seed[s]);
    if (p->seed_read[s]) (void)hipEventDestroy(p->seed_read[s]);
  }
  if (p->d_pass) (void)hipFree(p->d_pass);
  if (p->d_pass_chunk) (void)hipFree(p->d_pass_chunk);
  if (p->copy) (void)hipStreamDestroy(p->copy);
  delete p->pool;
  delete p;
  return FS_OK;
}

extern "C" int fs_plan_create(const fs_plan_desc* desc, fs_plan** out) {
  FS_REQUIRE(desc && out, "null pointer");
  const fs_plan_desc& d = *desc;
  FS_REQUIRE(d.N >= 1 && d.E >= 0 && d.C >= 1 && d.ld >= 64 && d.ld % 64 == 0, "bad sizes");
  FS_REQUIRE(d.h_n && d.d_phi && d.d_row_off && d.d_labels && d.d_W_g && d.d_W_out && d.d_loss_hist,
             "null pointer");
  *out = nullptr;
  fs_plan* p = new fs_plan();
  p->d = d;
  int64_t rows = 0;
  for (int j = 0; j < d.N; ++j) {
    if (d.h_n[j] < 0) {
      delete p;
      return fail(FS_EINVAL, "fs_plan_create: negative client size");
    }
    for (int e = 0; e < d.E; ++e) {
      p->n.push_back(d.h_n[j]);
      p->off.push_back((int64_t)d.E * rows + (int64_t)e * d.h_n[j]);
    }
    rows += d.h_n[j];
  }
  p->perm_len = std::max<int64_t>(1, (int64_t)d.E * rows);
  const int64_t P = (int64_t)p->n.size();
  for (int64_t v : p->n) p->max_n = std::max(p->max_n, v);
  {
    int64_t mx = 0;
    for (int j = 0; j < d.N; ++j) mx = std::max(mx, d.h_n[j]);
    p->max_client_steps = std::max<int64_t>(1, (int64_t)d.E * ((mx + d.B - 1) / std::max(1, d.B)));
  }
  // FS_PHASE_EVAL_DEFER: a parallel split launch that leaves CUs idle evaluates the previous
  // round's global model on them (fs_tuning.no_eval_fuse turns this off)
  if (d.d_phi_t && d.n_t > 0 && d.d_labels_t && d.d_eval_ws && d.C <= 16 && d.G > 1 && !d.chained) {
    if (!fs::tuning().no_eval_fuse) {
      const int idle = fs::split_idle_cus(d.N, d.C, d.B, d.ld, d.G, 0);
      p->fuse_E = (int)std::min<int64_t>(idle, (d.n_t + 15) / 16);
    }
  }
  hipError_t e = hipSuccess;
  for (int s = 0; s < 2 && e == hipSuccess; ++s) {
    if (!d.shuffle_device) {
      e = hipHostMalloc(reinterpret_cast<void**>(&p->h_perm[s]), sizeof(int32_t) * p->perm_len, hipHostMallocDefault);
    }
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p->d_perm[s]), sizeof(int32_t) * p->perm_len);
    // ordering-only events: no timestamps and no system-scope release when they complete (the
    // waits are device-side, and the host only needs the seed upload's completion, not the
    // visibility of device writes)
    const unsigned evf = hipEventDisableTiming | (unsigned)hipEventDisableSystemFence;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->uploaded[s], evf);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->consumed[s], evf);
  }
  if (d.shuffle_device) {
    // the seeds stay in pinned, coherent host memory that the shuffle kernel reads directly
    // (round 2, r02s2: no slower than a hipMemcpyAsync upload, and no copy on the side stream)
    p->seed_copy = false;
    for (int k = 0; k < fs_plan::SEED_SLOTS && e == hipSuccess; ++k) {
      e = hipHostMalloc(reinterpret_cast<void**>(&p->h_seed[k]), sizeof(int64_t) * std::max<int64_t>(1, P),
                        p->seed_copy ? hipHostMallocDefault : (hipHostMallocMapped | hipHostMallocCoherent));
      if (e == hipSuccess && !p->seed_copy)
        e = hipHostGetDevicePointer(reinterpret_cast<void**>(&p->h_seed_dev[k]), p->h_seed[k], 0);
      if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p->d_seed[k]), sizeof(int64_t) * std::max<int64_t>(1, P));
      if (e == hipSuccess) e = hipEventCreateWithFlags(&p->seed_read[k], hipEventDisableTiming | hipEventDisableSystemFence);
    }
  }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking);
  if (e == hipSuccess && d.shuffle_device && P > 0) {
    std::vector<int64_t> h(2 * P);
    std::copy(p->n.begin(), p->n.end(), h.begin());
    std::copy(p->off.begin(), p->off.end(), h.begin() + P);
    e = hipMalloc(reinterpret_cast<void**>(&p->d_pass), sizeof(int64_t) * 2 * P);
    if (e == hipSuccess) e = hipMemcpy(p->d_pass, h.data(), sizeof(int64_t) * 2 * P, hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    fs_plan_destroy(p);
    return hip_fail("fs_plan_create", e);
  }
  if (!d.shuffle_device) {
    const int nthreads =
        d.host_threads > 0 ? d.host_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    p->pool = new Pool(nthreads);
    int dev = 0;
    (void)hipGetDevice(&dev);
    p->coord = std::thread([p, dev] {
      (void)hipSetDevice(dev);
      coordinator(p);
    });
  }
  *out = p;
  return FS_OK;
}

// Device replay: upload the seeds and launch fs_randperm_device on the side stream.
static int device_shuffle(fs_plan* p, const int64_t* h_seeds, int t) {
  const int s = t & 1;
  const int64_t P = (int64_t)p->n.size();
  const int k = t % fs_plan::SEED_SLOTS;
  if (p->seed_pending[k]) FS_HIP(hipEventSynchronize(p->seed_read[k]), "fs_plan_shuffle");   // pinned seeds free
  std::memcpy(p->h_seed[k], h_seeds, sizeof(int64_t) * P);
  if (p->cons_recorded[s]) FS_HIP(hipStreamWaitEvent(p->copy, p->consumed[s], 0), "fs_plan_shuffle");
  // optionally also behind the latest local training (the other slot's consumer)
  if (p->d.shuffle_after_train && p->cons_recorded[s ^ 1])
    FS_HIP(hipStreamWaitEvent(p->copy, p->consumed[s ^ 1], 0), "fs_plan_shuffle");
  if (p->seed_copy)
    FS_HIP(hipMemcpyAsync(p->d_seed[k], p->h_seed[k], sizeof(int64_t) * P, hipMemcpyHostToDevice, p->copy),
           "fs_plan_shuffle");
  const int64_t* seeds = p->seed_copy ? p->d_seed[k] : p->h_seed_dev[k];
  // (no error word: p->max_n is the maximum of the plan's own pass sizes)
  const int rc = fs_randperm_device(seeds, p->d_pass, p->d_pass + P, P, p->max_n, p->d_perm[s], nullptr, p->copy);
  if (rc != FS_OK) return rc;
  FS_HIP(hipEventRecord(p->seed_read[k], p->copy), "fs_plan_shuffle");
  p->seed_pending[k] = true;
  FS_HIP(hipEventRecord(p->uploaded[s], p->copy), "fs_plan_shuffle");
  p->up_pending[s] = true;
  p->slot_round[s] = t;
  return FS_OK;
}

// Chunked device replay: the seeds of rounds cK .. cK+K-1 are collected in one pinned seed
// slot; one fs_randperm_device launch over all K*P passes fills shuffle slot c & 1.
extern "C" int fs_plan_set_shuffle_chunk(fs_plan* p, int rounds) {
  FS_REQUIRE(p && rounds >= 1 && rounds <= 64, "bad arguments");
  FS_REQUIRE(p->d.shuffle_device, "fs_plan_set_shuffle_chunk: device replay only");
  FS_REQUIRE(!p->seed_pending[0] && p->slot_round[0] < 0 && p->slot_round[1] < 0 && p->slot_chunk[0] < 0 &&
                 p->fill_chunk < 0,
             "fs_plan_set_shuffle_chunk: set before the first shuffle");
  if (rounds == p->chunk) return FS_OK;
  const int64_t P = (int64_t)p->n.size();
  const int64_t KP = std::max<int64_t>(1, (int64_t)rounds * P);
  for (int s = 0; s < 2; ++s) {
    FS_HIP(hipFree(p->d_perm[s]), "fs_plan_set_shuffle_chunk");
    p->d_perm[s] = nullptr;
    FS_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_perm[s]), sizeof(int32_t) * p->perm_len * rounds),
           "fs_plan_set_shuffle_chunk");
  }
  for (int k = 0; k < fs_plan::SEED_SLOTS; ++k) {
    FS_HIP(hipHostFree(p->h_seed[k]), "fs_plan_set_shuffle_chunk");
    FS_HIP(hipFree(p->d_seed[k]), "fs_plan_set_shuffle_chunk");
    p->h_seed[k] = nullptr;
    p->d_seed[k] = nullptr;
    FS_HIP(hipHostMalloc(reinterpret_cast<void**>(&p->h_seed[k]), sizeof(int64_t) * KP,
                         p->seed_copy ? hipHostMallocDefault : (hipHostMallocMapped | hipHostMallocCoherent)),
           "fs_plan_set_shuffle_chunk");
    if (!p->seed_copy)
      FS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&p->h_seed_dev[k]), p->h_seed[k], 0),
             "fs_plan_set_shuffle_chunk");
    FS_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_seed[k]), sizeof(int64_t) * KP), "fs_plan_set_shuffle_chunk");
  }
  if (p->d_pass_chunk) FS_HIP(hipFree(p->d_pass_chunk), "fs_plan_set_shuffle_chunk");
  p->d_pass_chunk = nullptr;
  if (P > 0) {
    std::vector<int64_t> h(2 * KP);
    for (int r = 0; r < rounds; ++r)
      for (int64_t i = 0; i < P; ++i) {
        h[r * P + i] = p->n[i];
        h[KP + r * P + i] = p->off[i] + (int64_t)r * p->perm_len;
      }
    FS_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_pass_chunk), sizeof(int64_t) * 2 * KP),
           "fs_plan_set_shuffle_chunk");
    FS_HIP(hipMemcpy(p->d_pass_chunk, h.data(), sizeof(int64_t) * 2 * KP, hipMemcpyHostToDevice),
           "fs_plan_set_shuffle_chunk");
  }
  p->chunk = rounds;
  return FS_OK;
}

// launch the shuffles of the collected rounds of chunk p->fill_chunk into slot (chunk & 1)
static int launch_chunk(fs_plan* p) {
  const int c = p->fill_chunk, nr = p->fill_rounds, K = p->chunk;
  const int s = c & 1, k = c % fs_plan::SEED_SLOTS;
  const int64_t P = (int64_t)p->n.size(), KP = std::max<int64_t>(1, (int64_t)K * P);
  // the slot's previous chunk (c - 2) released it after its last local training
  if (p->cons_recorded[s]) FS_HIP(hipStreamWaitEvent(p->copy, p->consumed[s], 0), "fs_plan_shuffle");
  if (P > 0) {
    if (p->seed_copy)
      FS_HIP(hipMemcpyAsync(p->d_seed[k], p->h_seed[k], sizeof(int64_t) * nr * P, hipMemcpyHostToDevice, p->copy),
             "fs_plan_shuffle");
    const int64_t* seeds = p->seed_copy ? p->d_seed[k] : p->h_seed_dev[k];
    // (no error word: the plan's max_n is the maximum of its own pass sizes, so no pass exceeds it)
    const int rc = fs_randperm_device(seeds, p->d_pass_chunk, p->d_pass_chunk + KP, nr * P, p->max_n, p->d_perm[s],
                                      nullptr, p->copy);
    if (rc != FS_OK) return rc;
  }
  FS_HIP(hipEventRecord(p->seed_read[k], p->copy), "fs_plan_shuffle");
  p->seed_pending[k] = true;
  FS_HIP(hipEventRecord(p->uploaded[s], p->copy), "fs_plan_shuffle");
  p->up_pending[s] = true;
  p->slot_chunk[s] = c;
  p->slot_nrounds[s] = nr;
  p->fill_chunk = -1;
  p->fill_rounds = 0;
  return FS_OK;
}

static int chunk_shuffle(fs_plan* p, const int64_t* h_seeds, int t) {
  const int K = p->chunk, c = t / K, r = t % K;
  const int64_t P = (int64_t)p->n.size();
  FS_REQUIRE(r == (p->fill_chunk == c ? p->fill_rounds : 0) && (r > 0 || p->fill_chunk < 0),
             "rounds must be prepared in order");
  if (r == 0) {
    const int k = c % fs_plan::SEED_SLOTS;
    if (p->seed_pending[k]) FS_HIP(hipEventSynchronize(p->seed_read[k]), "fs_plan_shuffle");   // seed slot free
    p->fill_chunk = c;
    p->fill_rounds = 0;
  }
  std::memcpy(p->h_seed[c % fs_plan::SEED_SLOTS] + (int64_t)r * P, h_seeds, sizeof(int64_t) * P);
  ++p->fill_rounds;
  return r == K - 1 ? launch_chunk(p) : FS_OK;
}

// Timing events for measurement (bench.py's per-launch durations): timestamps, but no
// system-scope release when recorded (hipEventDisableSystemFence) -- a default timing event
// between two kernels of a round cost ~3.5 us of GPU idle each at config 2 (r02s2z).
extern "C" int fs_timer_create(void** ev) {
  FS_REQUIRE(ev, "null pointer");
  hipEvent_t e = nullptr;
  FS_HIP(hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence), "fs_timer_create");
  *ev = e;
  return FS_OK;
}
extern "C" int fs_timer_record(void* ev, void* stream) {
  FS_REQUIRE(ev, "null pointer");
  FS_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), reinterpret_cast<hipStream_t>(stream)), "fs_timer_record");
  return FS_OK;
}
extern "C" int fs_timer_elapsed_ms(void* start, void* end, float* ms) {
  FS_REQUIRE(start && end && ms, "null pointer");
  FS_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(end)), "fs_timer_elapsed_ms");
  FS_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(end)),
         "fs_timer_elapsed_ms");
  return FS_OK;
}
extern "C" int fs_timer_destroy(void* ev) {
  if (ev) FS_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)), "fs_timer_destroy");
  return FS_OK;
}

extern "C" int fs_plan_eval_blocks(const fs_plan* p) {
  FS_REQUIRE(p, "bad arguments");
  return p->fuse_E;
}

extern "C" int fs_plan_shuffle_flush(fs_plan* p) {
  FS_REQUIRE(p, "bad arguments");
  return (p->chunk > 1 && p->fill_chunk >= 0) ? launch_chunk(p) : FS_OK;
}

// Prepare round t's shuffles: device replay is enqueued here; a host replay job is queued
// for the coordinator thread and this returns at once.
extern "C" int fs_plan_shuffle(fs_plan* p, const int64_t* h_seeds, int t) {
  FS_REQUIRE(p && (h_seeds || p->n.empty()) && t >= 0, "bad arguments");
  if (p->d.shuffle_device) {
    if (p->chunk > 1) return chunk_shuffle(p, h_seeds, t);
    if (p->n.empty()) {
      p->slot_round[t & 1] = t;
      return FS_OK;
    }
    return device_shuffle(p, h_seeds, t);
  }
  {
    std::lock_guard<std::mutex> lk(p->m);
    if (p->job_status != FS_OK) return fail(p->job_status, p->job_error);
    p->jobs.emplace_back(t, std::vector<int64_t>(h_seeds, h_seeds + p->n.size()));
  }
  p->cv.notify_all();
  return FS_OK;
}

static int run_shuffle_job(fs_plan* p, const int64_t* h_seeds, int t) {
  const int s = t & 1;
  if (p->up_pending[s]) FS_HIP(hipEventSynchronize(p->uploaded[s]), "fs_plan_shuffle");   // pinned slot free
  int32_t* out = p->h_perm[s];
  const std::function<void(int64_t)> one = [&](int64_t i) {
    replay_randperm((uint64_t)h_seeds[i], p->n[i], out + p->off[i]);
  };
  p->pool->run((int64_t)p->n.size(), one);
  // the device slot is rewritten only after the local training that read it has finished
  if (p->cons_recorded[s]) FS_HIP(hipStreamWaitEvent(p->copy, p->consumed[s], 0), "fs_plan_shuffle");
  FS_HIP(hipMemcpyAsync(p->d_perm[s], out, sizeof(int32_t) * p->perm_len, hipMemcpyHostToDevice, p->copy),
         "fs_plan_shuffle");
  FS_HIP(hipEventRecord(p->uploaded[s], p->copy), "fs_plan_shuffle");
  p->up_pending[s] = true;
  std::lock_guard<std::mutex> lk(p->m);
  p->slot_round[s] = t;
  return FS_OK;
}

// the deferred evaluation of round p->eval_pending as a launch of its own
static int flush_eval(fs_plan* p, hipStream_t st) {
  if (p->eval_pending < 0) return FS_OK;
  const fs_plan_desc& d = p->d;
  const int te = p->eval_pending;
  p->eval_pending = -1;
  return fs_eval(d.d_phi_t, d.ld, d.d_labels_t, d.n_t, d.d_W_g, d.C, d.d_eval_hist + 2 * (int64_t)te, d.d_eval_ws, st);
}

// ABI 15: complete every evaluation this plan still holds -- a deferred one
// not yet carried by a TRAIN launch (as its own fs_eval launch) and a fused one whose finaliser
// waits for the next AGGREGATE -- so d_eval_hist is final once `stream` reaches this point.
extern "C" int fs_plan_eval_flush(fs_plan* p, void* stream) {
  FS_REQUIRE(p, "bad arguments");
  const fs_plan_desc& d = p->d;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (p->fin_pending >= 0) {
    const fs::EvalFinalize f{d.d_eval_ws, p->fuse_E, (int)d.n_t, d.d_eval_hist + 2 * (int64_t)p->fin_pending};
    p->fin_pending = -1;
    const int rc = fs::eval_finalize_launch(f.part, f.nb, f.n, f.out, st);
    if (rc != FS_OK) return rc;
  }
  return flush_eval(p, st);
}

extern "C" int fs_plan_round(fs_plan* p, int t, float lr, int phases, const float* d_p_override, void* stream) {
  FS_REQUIRE(p && t >= 0, "bad arguments");
  const fs_plan_desc& d = p->d;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int s = t & 1;
  // a deferred evaluation rides on this TRAIN launch (it reads W_g before the launch
  // rewrites nothing but W_out); anything else that follows it runs it on its own first
  fs::FuseEval fuse{d.d_phi_t, d.d_labels_t, (int)d.n_t, p->fuse_E, d.d_eval_ws};
  auto fin_of = [&](int te) { return fs::EvalFinalize{d.d_eval_ws, p->fuse_E, (int)d.n_t, d.d_eval_hist + 2 * (int64_t)te}; };
  // a finaliser left by an earlier TRAIN call rides on this call's aggregation -- unless this
  // call trains (its fused evaluation rewrites the partials) or does not aggregate: then first
  if (p->fin_pending >= 0 && ((phases & FS_PHASE_TRAIN) || !(phases & FS_PHASE_AGGREGATE))) {
    const fs::EvalFinalize f = fin_of(p->fin_pending);
    p->fin_pending = -1;
    const int rc = fs::eval_finalize_launch(f.part, f.nb, f.n, f.out, st);
    if (rc != FS_OK) return rc;
  }
  const bool fused = (phases & FS_PHASE_TRAIN) && p->eval_pending >= 0 && p->fuse_E > 0;
  if (p->eval_pending >= 0 && !fused) {
    const int rc = flush_eval(p, st);
    if (rc != FS_OK) return rc;
  }
  const int t_eval = p->eval_pending;
  if ((phases & FS_PHASE_TRAIN) && p->chunk > 1) {
    const int K = p->chunk, c = t / K, r = t % K, sc = c & 1;
    // a partly collected chunk (the last rounds of a run) is launched when first needed
    if (p->slot_chunk[sc] != c && p->fill_chunk == c) {
      const int rc = launch_chunk(p);
      if (rc != FS_OK) return rc;
    }
    if (p->slot_chunk[sc] != c || r >= p->slot_nrounds[sc])
      return fail(FS_EINVAL, "fs_plan_round: shuffles of this round were not prepared");
    if (p->slot_waited[sc] != c) {                 // once per chunk
      FS_HIP(hipStreamWaitEvent(st, p->uploaded[sc], 0), "fs_plan_round");
      p->slot_waited[sc] = c;
    }
    const int rc = fs::local_train(d.d_phi, d.ld, d.d_row_off, d.d_labels, p->d_perm[sc] + (int64_t)r * p->perm_len,
                                  d.d_order, d.N, d.C, d.B, d.E, lr, d.mu, d.prox, d.lam, d.reg, d.chained, d.d_W_g,
                                  d.d_W_out, d.d_loss_hist + (int64_t)t * d.N, d.G, d.d_ws, d.ws_bytes, st,
                                  p->max_client_steps, fused ? &fuse : nullptr);
    if (rc != FS_OK) return rc;
    if (r == p->slot_nrounds[sc] - 1) {            // the chunk's last round releases the slot
      FS_HIP(hipEventRecord(p->consumed[sc], st), "fs_plan_round");
      p->cons_recorded[sc] = true;
    }
  } else if (phases & FS_PHASE_TRAIN) {
    {
      // wait for this round's shuffle job (normally finished long ago)
      std::unique_lock<std::mutex> lk(p->m);
      p->done.wait(lk, [&] {
        if (p->job_status != FS_OK || p->slot_round[s] == t) return true;
        for (auto& j : p->jobs) if (j.first == t) return false;
        return true;                               // never queued
      });
      if (p->job_status != FS_OK) return fail(p->job_status, p->job_error);
      if (p->slot_round[s] != t) return fail(FS_EINVAL, "fs_plan_round: shuffles of this round were not prepared");
    }
    FS_HIP(hipStreamWaitEvent(st, p->uploaded[s], 0), "fs_plan_round");
    const int rc = fs::local_train(d.d_phi, d.ld, d.d_row_off, d.d_labels, p->d_perm[s], d.d_order, d.N, d.C, d.B,
                                   d.E, lr, d.mu, d.prox, d.lam, d.reg, d.chained, d.d_W_g, d.d_W_out,
                                   d.d_loss_hist + (int64_t)t * d.N, d.G, d.d_ws, d.ws_bytes, st,
                                   p->max_client_steps, fused ? &fuse : nullptr);
    if (rc != FS_OK) return rc;
    FS_HIP(hipEventRecord(p->consumed[s], st), "fs_plan_round");
    p->cons_recorded[s] = true;
  }
  // the fused evaluation's finaliser rides on the next aggregation launch, this call's or a later
  // call's (the two are independent: the partials of round t_eval's W_g vs this round's W_out;
  // the FedAvg driver's TRAIN and AGGREGATE | EVAL calls of a round: one launch fewer per round)
  if (fused) {
    p->eval_pending = -1;
    p->fin_pending = t_eval;
  }
  if (phases & FS_PHASE_AGGREGATE) {
    const float* pw = d_p_override ? d_p_override : d.d_p;
    FS_REQUIRE(pw, "no mixture weights");
    const int64_t len = (int64_t)d.C * d.ld;
    const fs::EvalFinalize fin = fin_of(p->fin_pending);
    const bool with_fin = p->fin_pending >= 0;
    p->fin_pending = -1;
    const int rc = fs::aggregate_launch(d.d_W_out, len, pw, d.N, len, d.d_W_g, d.d_agg_ws, d.agg_ws_floats,
                                        d.agg_chunks, with_fin ? &fin : nullptr, st);
    if (rc != FS_OK) return rc;
  }
  // (a finaliser still pending here is launched by the next fs_plan_round call -- any call that
  // trains or does not aggregate runs it first; results are read after such a call)
  if (phases & FS_PHASE_EVAL) {
    FS_REQUIRE(d.d_phi_t && d.d_labels_t && d.d_eval_hist && d.d_eval_ws, "no test set");
    if ((phases & FS_PHASE_EVAL_DEFER) && p->fuse_E > 0) {
      p->eval_pending = t;                         // evaluated by the next TRAIN launch
      return FS_OK;
    }
    const int rc = fs_eval(d.d_phi_t, d.ld, d.d_labels_t, d.n_t, d.d_W_g, d.C, d.d_eval_hist + 2 * (int64_t)t,
                           d.d_eval_ws, stream);
    if (rc != FS_OK) return rc;
  }
  return FS_OK;
}
