// Host side of the C-ABI: error plumbing and the DataLoader shuffle replay.
//
// fs_randperm_batch reproduces, bit for bit, the permutation that
// torch.utils.data.RandomSampler draws for one shuffled DataLoader pass
// (/root/reference/functions/tools.py:179, 220; /root/reference/exp.py:99):
//   g = torch.Generator(); g.manual_seed(seed); torch.randperm(n, generator=g)
// torch's CPU generator is MT19937 seeded with (uint32)seed and its randperm is a
// forward Fisher-Yates taking z = mt() % (n - i) (checked
// against torch in tests/test_rng.py).  Passes are independent, so they are spread
// over host threads.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fedsim.h"
#include "mt_replay.h"

namespace fs {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

static std::mutex g_tune_m;
static fs_tuning g_tune{};
// fs_set_thread_tuning: an override for the launches this host thread enqueues
static thread_local bool t_tune_set = false;
static thread_local fs_tuning t_tune{};

fs_tuning tuning() {
  if (t_tune_set) return t_tune;
  std::lock_guard<std::mutex> lk(g_tune_m);
  return g_tune;
}

static int check_tuning(const fs_tuning* t, const char* fn) {
  if (t && (t->mix_prefetch < -1 || t->mix_prefetch > 224 || t->mix_prefetch_lead < 0))
    return fail(FS_EINVAL, std::string(fn) + ": mix_prefetch must be in [-1, 224], mix_prefetch_lead >= 0");
  if (t && (t->train_form < 0 || t->train_form > 2))
    return fail(FS_EINVAL, std::string(fn) + ": train_form must be 0, 1 or 2");
  if (t && (t->split_early < -1 || t->split_early > 0))
    return fail(FS_EINVAL, std::string(fn) + ": split_early must be -1 or 0");
  if (t && t->mix_qmc_lane_clients != 0 && t->mix_qmc_lane_clients != 4 && t->mix_qmc_lane_clients != 8)
    return fail(FS_EINVAL, std::string(fn) + ": mix_qmc_lane_clients must be 0, 4 or 8");
  if (t && (t->mix_quad_loaders < -1 || t->mix_quad_loaders > 0))
    return fail(FS_EINVAL, std::string(fn) + ": mix_quad_loaders must be -1 or 0");
  if (t && (t->split_teams < -1 || t->split_teams > 1))
    return fail(FS_EINVAL, std::string(fn) + ": split_teams must be -1, 0 or 1");
  if (t && (t->mix_poll_delay < -1 || t->mix_poll_delay > 4096))
    return fail(FS_EINVAL, std::string(fn) + ": mix_poll_delay must be in [-1, 4096]");
  if (t && (t->split_poll_delay < -1 || t->split_poll_delay > 4096))
    return fail(FS_EINVAL, std::string(fn) + ": split_poll_delay must be in [-1, 4096]");
  if (t && (t->split_pipe < -1 || t->split_pipe > 1))
    return fail(FS_EINVAL, std::string(fn) + ": split_pipe must be -1, 0 or 1");
  if (t && (t->split_dbuf < -1 || t->split_dbuf > 1))
    return fail(FS_EINVAL, std::string(fn) + ": split_dbuf must be -1, 0 or 1");
  if (t && (t->split_mb < -1 || t->split_mb > 1))
    return fail(FS_EINVAL, std::string(fn) + ": split_mb must be -1, 0 or 1");
  return FS_OK;
}

}  // namespace fs

extern "C" int fs_abi_version(void) { return FS_ABI_VERSION; }

extern "C" int64_t fs_tuning_size(void) { return (int64_t)sizeof(fs_tuning); }

extern "C" int fs_set_tuning(const fs_tuning* t) {
  if (int rc = fs::check_tuning(t, "fs_set_tuning")) return rc;
  std::lock_guard<std::mutex> lk(fs::g_tune_m);
  fs::g_tune = t ? *t : fs_tuning{};
  return FS_OK;
}

extern "C" int fs_set_thread_tuning(const fs_tuning* t) {
  if (int rc = fs::check_tuning(t, "fs_set_thread_tuning")) return rc;
  fs::t_tune_set = t != nullptr;
  fs::t_tune = t ? *t : fs_tuning{};
  return FS_OK;
}

extern "C" int fs_get_tuning(fs_tuning* t) {
  if (!t) return fs::fail(FS_EINVAL, "fs_get_tuning: null pointer");
  *t = fs::tuning();
  return FS_OK;
}

extern "C" int fs_get_process_tuning(fs_tuning* t) {
  if (!t) return fs::fail(FS_EINVAL, "fs_get_process_tuning: null pointer");
  std::lock_guard<std::mutex> lk(fs::g_tune_m);
  *t = fs::g_tune;
  return FS_OK;
}

extern "C" int fs_get_thread_tuning(fs_tuning* t) {
  if (!t) return fs::fail(FS_EINVAL, "fs_get_thread_tuning: null pointer");
  *t = fs::t_tune_set ? fs::t_tune : fs_tuning{};
  return fs::t_tune_set ? 1 : 0;
}

extern "C" const char* fs_last_error(void) { return fs::g_last_error.c_str(); }

extern "C" int fs_randperm_batch(const int64_t* h_seeds, const int64_t* h_n, const int64_t* h_off, int64_t npasses,
                                 int32_t* h_out, int nthreads) {
  if (npasses < 0 || (npasses > 0 && (!h_seeds || !h_n || !h_off || !h_out)))
    return fs::fail(FS_EINVAL, "fs_randperm_batch: bad arguments");
  for (int64_t i = 0; i < npasses; ++i)
    if (h_n[i] < 0 || h_n[i] >= (int64_t)1 << 31) return fs::fail(FS_EINVAL, "fs_randperm_batch: n out of range");
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  int64_t total = 0;
  for (int64_t i = 0; i < npasses; ++i) total += h_n[i];
  if (nthreads == 1 || npasses <= 1 || total < (1 << 15)) {
    for (int64_t i = 0; i < npasses; ++i) fs::replay_randperm((uint64_t)h_seeds[i], h_n[i], h_out + h_off[i]);
    return FS_OK;
  }
  nthreads = (int)std::min<int64_t>(nthreads, npasses);
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= npasses) return;
      fs::replay_randperm((uint64_t)h_seeds[i], h_n[i], h_out + h_off[i]);
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(nthreads - 1);
  for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  return FS_OK;
}
