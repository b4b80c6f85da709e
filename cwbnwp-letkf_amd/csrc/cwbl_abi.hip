// cwbl_abi.hip — C ABI of the LETKF analysis core (include/cwb_letkf_core.h).
//
// Host orchestration of one variable, mirroring letkf_driver (module_letkf_core.f90:59-297):
//   build_tree x2        -> host kdtree2-compatible build, upload (kdtree_build.cpp)
//   (point-independent)  -> obs_prep_kernel per obs type (QC / mean / spread columns)
//   points :209-240      -> batches of {search_kernel, solve_kernel<KP>} on one HIP stream
// The library owns its device buffers between cwbl_set_obs and cwbl_finalize; host arrays
// handed in are copied inside the call.  There is no CPU fallback: without a gfx950 device
// every compute entry point fails with CWBL_ERR_NO_DEVICE.
#include "../../include/cwb_letkf_core.h"
#include "cwbl_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace cwbl {
namespace {

std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(CWBL_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                  __FILE__, __LINE__);                                                     \
  } while (0)

// grow-only device buffer
struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// grow-only page-locked host buffer (bounce slots of pageable host slabs)
struct PinBuf {
  void *p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// A few persistent host threads for the bounce copies: run(n, fn) calls fn(0..n-1) spread
// over the threads and the caller, and returns when all calls are done.
class HostPool {
 public:
  ~HostPool() { stop(); }
  void run(int n, const std::function<void(int)> &fn) {
    if (n <= 0) return;
    start();
    {
      std::unique_lock<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      busy_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
    th_.clear();
    quit_ = false;
  }

 private:
  void start() {
    if (!th_.empty()) return;
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    int nt = (int)std::min(15u, hw - 1);  // + the calling thread: at most 16
    if (const char *e = std::getenv("OMP_NUM_THREADS"))
      nt = std::max(0, std::min(nt, std::atoi(e) - 1));
    // a new worker starts at the current generation: stop() of an earlier pool raised gen_,
    // and a worker starting from 0 would run a pass no run() handed out (and decrement
    // busy_ twice)
    unsigned long g;
    {
      std::lock_guard<std::mutex> lk(mu_);
      g = gen_;
    }
    for (int i = 0; i < nt; ++i) th_.emplace_back([this, g] { loop(g); });
  }
  void work() {
    for (;;) {
      int i;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!fn_ || next_ >= n_) return;
        i = next_++;
      }
      (*fn_)(i);
    }
  }
  void loop(unsigned long seen) {
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (quit_) return;
      }
      work();
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--busy_ == 0) done_.notify_all();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)> *fn_ = nullptr;
  int n_ = 0, next_ = 0, busy_ = 0;
  unsigned long gen_ = 0;
  bool quit_ = false;
};

struct ObsType {
  int family = 0, type_id = 0, nvar = 1, nobs = 0;
  std::vector<float> xyz;   // host copy (3,nobs) for tree builds
  DevBuf obs, error, hdxb, qc;
};

// One k-d tree of an obs type and its column tables.  The tree depends only on the obs
// coordinates and the normalisation (hclr, vclr, dimension), so it is kept across
// cwbl_analyze_var calls of one obs set; the column tables are rebuilt per call (they
// depend on the variable's QC parameters).
struct TreeBufs {
  int entry = -1, dim = 0, depth = 0;
  int bin_div_opt = 0;  // CWBL_OPT_BIN_DIV the bins were built under
  float hinv = 0.0f, vinv = 0.0f;
  DevBuf nodes, rdata, ind, col_bg, col_omm, col_err, col_ok;
  DevBuf bxyz, bstart;  // uniform bins of the same coordinates (search_binned_kernel)
  HostTree host;
  HostBins bins;
  void release() {
    nodes.release(); rdata.release(); ind.release(); col_bg.release();
    col_omm.release(); col_err.release(); col_ok.release(); bxyz.release(); bstart.release();
  }
};

enum KernelId {
  KT_SEARCH_BINNED, KT_SEARCH_FLAGGED, KT_SEARCH_TREE, KT_ASSEMBLE_RECORD, KT_SOLVE_TQ40,
  KT_BIG_HANDOFF, KT_TQB_TAIL, KT_SOLVE_TQ, KT_SOLVE_TQ_BIG, KT_SOLVE_JACOBI, KT_TUNE_Q,
  KT_COUNT
};
struct KTime { long long launches = 0, points = 0; double ms = 0.0; };

struct State {
  bool inited = false;
  int k = 0, kp = 0, device = 0, wf = 0, q1_mode = 0;
  int kp_natural = 0;  // smallest compiled KP >= k (kp: the one the options select)
  float norain = -5.0f;
  size_t ws_bytes = size_t(2) << 30;
  hipStream_t stream = nullptr;
  std::vector<ObsType> obs;  // gts entries first (family 0), then radar (family 1)
  bool have_obs = false;
  std::vector<std::unique_ptr<TreeBufs>> tree_cache;  // trees of the current obs set
  DevBuf tdesc, nbr_cnt, nbr_idx, info, stats;
  DevBuf nbr_cnt2, nbr_idx2;                          // second list buffer (search overlap)
  hipStream_t sstream = nullptr;                      // neighbour searches of later batches
  std::vector<hipEvent_t> cevents;                    // ordering events of the host copies
  int lead_div = 0;                                   // first batch = npts / lead_div (0: off)
  bool serial_search = false;                         // CWBL_DEBUG_SERIAL=1: searches on S.stream
  // Points per search/solve batch.  Measured on C2 (one GPU, ms per variable): 40 k 113,
  // 70 k 110, 100 k 108, 150 k 107, 200 k 106, 500 k 109; and on an eighth of the grid (a
  // rank of the 8-GPU run): 14.7-15.0 up to 150 k, 15.3 at 200 k, 16.6 at 285 k.  Smaller
  // batches keep each batch's lists and hand-off records nearer the caches and overlap
  // more of the search; below ~70 k the per-batch fixed costs win.
  long long max_batch = 160000;
  bool max_batch_set = false;
  // one-stream path: the per-point info (solved, p) of a window of up to info_window points
  // is reduced once per window (a reduction kernel per batch cost the C2 step ~0.5 ms)
  long long info_window = 1LL << 25;  // 256 MB of int2 (CWBL_OPT_INFO_WINDOW)                         // CWBL_OPT_MAX_BATCH given: no ~6-batch rule
  DevBuf sx, sy, salt, svar;                          // slab staging (host-memory calls)
  DevBuf bcol, byo, byb, bxb, bxa, bev, btri;         // solve_batch staging (btri: T per point)
  DevBuf qxyz, qnf, qidx, qr2;                        // search staging
  DevBuf quad;                                        // x^-1/2 quadrature tables
  DevBuf wsa;                                         // hand-off records (split KP=40 path)
  DevBuf flags;                                       // binned search: flagged points (+ count)
  bool binned = true;                                 // CWBL_OPT_SEARCH = 1: k-d tree search only
  int bin_div = 0;  // CWBL_OPT_BIN_DIV: bin side = radius / bin_div (0: by density, bin_div_for)
  bool pageable_register = true;                      // CWBL_OPT_PAGEABLE = 1: bounce slots
  bool jacobi = false;                                // CWBL_OPT_SOLVER = 1: Jacobi eigen path
  int tq4 = 1;  // CWBL_OPT_SPLIT40: KP=40 solve 0 = one kernel, else assembly record + solve_tq40
  long long tq4_sub = 0;                              // CWBL_TQ4_SUB: record batch (points)
  bool big_split = true;                              // big_path 1: hand-off + one-wave tail
  long long big_sub = 98304;                          // CWBL_OPT_BIG_BATCH: k > 64 sub-batch
  std::vector<hipEvent_t> events;
  hipStream_t h2d = nullptr, d2h = nullptr;           // host-memory slab copies (pipelined)
  hipStream_t caller_stream = nullptr;                // cwbl_set_stream (null: legacy stream)
  hipEvent_t order_ev = nullptr;                      // order_after_caller
  // cwbl_set_kernel_timing: every solve/search launch of cwbl_analyze_var bracketed by a HIP
  // event pair on the stream it runs on; summed per kernel after the call's final sync
  bool ktiming = false;
  KTime ktime[KT_COUNT];
  std::vector<hipEvent_t> kevents;
  int kev_used = 0;
  struct KPend { int id; hipEvent_t e0, e1; long long pts; };
  std::vector<KPend> kpend;
  size_t handoff_budget = 0;                          // bytes for the k > 64 hand-off records
  // pageable host slabs: each batch's var columns go through page-locked bounce slots (two
  // in, two out), filled and drained by a few host threads while the GPU runs other batches
  static constexpr int kSlots = 3;
  PinBuf pin_in[kSlots], pin_out[kSlots];
  HostPool pool;
};

State S;

float search_r2() {
  const float gc1999 = 2.0f * std::sqrt(10.0f / 3.0f);  // module_param.f90:116
  return gc1999 * gc1999;                               // module_localization.f90:202
}

bool is_gts_assimilated(int id) {  // module_localization.f90:59-72
  return id == CWBL_GTS_SYNOP || id == CWBL_GTS_METAR || id == CWBL_GTS_SHIPS ||
         id == CWBL_GTS_SOUND || id == CWBL_GTS_GPSPW;
}

int tree_depth(const HostTree &t, int node = 0) {
  if (t.nodes.empty()) return 0;
  int depth = 0;
  // iterative DFS over (node, level)
  std::vector<std::pair<int, int>> st{{node, 1}};
  while (!st.empty()) {
    auto [nd, lv] = st.back();
    st.pop_back();
    depth = std::max(depth, lv);
    if (t.nodes[nd].cut_dim >= 0) {
      st.push_back({t.nodes[nd].left, lv + 1});
      st.push_back({t.nodes[nd].right, lv + 1});
    }
  }
  return depth;
}

// copy an array given by the caller (host or device) into a library device buffer
hipError_t stage(DevBuf &dst, const void *src, size_t bytes, int memory) {
  hipError_t e = dst.ensure(bytes);
  if (e != hipSuccess || bytes == 0) return e;
  return hipMemcpyAsync(dst.p, src, bytes,
                        memory == CWBL_MEM_DEVICE ? hipMemcpyDeviceToDevice
                                                  : hipMemcpyHostToDevice,
                        S.stream);
}

hipError_t cevent(int i, hipEvent_t *out) {  // ordering events (timing off)
  while ((int)S.cevents.size() <= i) {
    hipEvent_t e;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) return r;
    S.cevents.push_back(e);
  }
  *out = S.cevents[i];
  return hipSuccess;
}

hipError_t event(int i, hipEvent_t *out) {
  while ((int)S.events.size() <= i) {
    hipEvent_t e;
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) return r;
    S.events.push_back(e);
  }
  *out = S.events[i];
  return hipSuccess;
}

float elapsed(int a, int b) {
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, S.events[a], S.events[b]) != hipSuccess) return 0.0f;
  return ms;
}

// Kernel timing (cwbl_set_kernel_timing): kt_begin records the first event of a launch's
// pair on its stream (-1 when timing is off), kt_end the second, queued for kt_collect.
hipError_t kt_event(int i, hipEvent_t *out) {
  while ((int)S.kevents.size() <= i) {
    hipEvent_t e;
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) return r;
    S.kevents.push_back(e);
  }
  *out = S.kevents[i];
  return hipSuccess;
}

hipError_t kt_begin(hipStream_t s, int *ev) {
  *ev = -1;
  if (!S.ktiming) return hipSuccess;
  hipEvent_t e;
  hipError_t r = kt_event(S.kev_used, &e);
  if (r != hipSuccess) return r;
  *ev = S.kev_used;
  S.kev_used += 2;
  return hipEventRecord(e, s);
}

hipError_t kt_end(hipStream_t s, int ev, int id, long long pts) {
  if (ev < 0) return hipSuccess;
  hipEvent_t e;
  hipError_t r = kt_event(ev + 1, &e);
  if (r != hipSuccess) return r;
  S.kpend.push_back({id, S.kevents[ev], e, pts});
  return hipEventRecord(e, s);
}

// Two launches back to back on one stream between events the call records anyway (e0 before
// the first, e1 after the second): one more event between them times both.  Each event
// between two kernels costs the stream ~5 us (r4: 4 per C2 batch were 0.9% of the step).
hipError_t kt_pair(hipStream_t s, hipEvent_t e0, int id0, long long pts0, hipEvent_t e1,
                   int id1, long long pts1, const std::function<hipError_t()> &first,
                   const std::function<hipError_t()> &second) {
  hipError_t r = first();
  if (r != hipSuccess) return r;
  if (S.ktiming) {
    hipEvent_t mid;
    r = kt_event(S.kev_used++, &mid);
    if (r != hipSuccess) return r;
    r = hipEventRecord(mid, s);
    if (r != hipSuccess) return r;
    S.kpend.push_back({id0, e0, mid, pts0});
    S.kpend.push_back({id1, mid, e1, pts1});
  }
  return second();
}

void kt_collect() {  // after the call's final synchronisation
  for (const State::KPend &p : S.kpend) {
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, p.e0, p.e1) != hipSuccess) continue;
    KTime &t = S.ktime[p.id];
    t.launches += 1;
    t.points += p.pts;
    t.ms += ms;
  }
  S.kpend.clear();
  S.kev_used = 0;
}

std::string kernel_name(int id) {
  const std::string kp = std::to_string(S.kp);
  switch (id) {
    case KT_SEARCH_BINNED: return "search_binned_kernel";
    case KT_SEARCH_FLAGGED: return "search_kernel<FlagQuery>";
    case KT_SEARCH_TREE: return "search_kernel<SlabQuery>";
    case KT_ASSEMBLE_RECORD: return "assemble_record_kernel<" + std::to_string(kRecordWaves) + ">";
    case KT_SOLVE_TQ40: return "solve_tq40_kernel<" + kp + ", 0>";
    case KT_BIG_HANDOFF:
      return S.kp == 128 ? "solve_tq_rows_kernel<128, 64>"
                         : "solve_tq_big_kernel<" + kp + ", false, " +
                               std::to_string(big_split_j0(S.kp)) + ">";
    case KT_TQB_TAIL:
      return "solve_tqb_tail_kernel<" + kp + ", " + std::to_string(big_split_j0(S.kp)) +
             (S.kp == 128 ? ", 3>" : ", 2>");
    case KT_SOLVE_TQ: return "solve_tq_kernel<" + kp + ", false>";
    case KT_SOLVE_TQ_BIG: return "solve_tq_big_kernel<" + kp + ", false>";
    case KT_SOLVE_JACOBI: return "solve_kernel<" + kp + ", false>";
    case KT_TUNE_Q: return "tune_q_kernel";
  }
  return "?";
}

// page-locked (hipHostMalloc'd or hipHostRegister'ed) host memory: DMA-able as it is
bool host_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// k rows of nb floats between a member-slowest host slab (row pitch L) and a packed slot
double g_bounce_ms = 0.0;  // host time in the bounce copies of the current call
void bounce_rows(HostPool &pool, float *slot, float *var, long long L, long long g0, int nb,
                 int k, bool to_slot) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t row = (size_t)nb * 4;
  pool.run(k, [&](int m) {
    float *h = var + (size_t)m * L + g0, *b = slot + (size_t)m * nb;
    if (to_slot) std::memcpy(b, h, row);
    else std::memcpy(h, b, row);
  });
  g_bounce_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int require_device() {
  if (!S.inited) return fail(CWBL_ERR_STATE, "cwbl_init has not been called");
  return CWBL_OK;
}

// The library's streams are non-blocking: they are not ordered after work the caller has
// queued on its own stream.  Every entry point that reads or writes caller device memory
// therefore first makes the library's stream wait for an event recorded on the caller's
// stream (cwbl_set_stream; the legacy null stream by default), so device buffers may be
// passed as soon as their producers have been *queued* there.  Only that stream is waited
// for: unrelated streams of the process (another rank's collectives, other compute) are not
// (host-memory calls need no wait: the caller's host arrays are complete when the call is
// made).
hipError_t order_after_caller() {
  if (!S.order_ev) {
    hipError_t e = hipEventCreateWithFlags(&S.order_ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  hipError_t e = hipEventRecord(S.order_ev, S.caller_stream);
  if (e != hipSuccess) return e;
  return hipStreamWaitEvent(S.stream, S.order_ev, 0);
}

// Bin side r / div for the uniform-bin search: r/2 by default; r/4 where the obs are dense
// (more than 24 per r/2 cell on average over the set's bounding box: the finer cells trim
// the per-row runs closer to the ball).  r4 A/B: C5 (49 per r/2 cell) 15.95 M pts/s at r/2,
// 16.04 at r/3, 16.19 at r/4; C2 (~11 per cell) 59.4 / 58.9 / 58.6.  CWBL_OPT_BIN_DIV forces it.
int bin_div_for(const HostTree &t, int dim) {
  if (S.bin_div > 0) return S.bin_div;
  const int n = t.n;
  if (n == 0) return 2;
  float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  bool seen = false;
  for (int i = 0; i < n; ++i) {
    const float *d = &t.rdata[4 * (size_t)i];
    if (!std::isfinite(d[0]) || !std::isfinite(d[1]) || (dim == 3 && !std::isfinite(d[2]))) continue;
    for (int c = 0; c < dim; ++c) {
      lo[c] = seen ? std::min(lo[c], d[c]) : d[c];
      hi[c] = seen ? std::max(hi[c], d[c]) : d[c];
    }
    seen = true;
  }
  const double h = 0.5 * std::sqrt((double)search_r2());
  double cells = 1.0;
  for (int c = 0; c < dim; ++c) cells *= std::max(1.0, ((double)hi[c] - (double)lo[c]) / h);
  return (double)n / cells > 24.0 ? 4 : 2;
}

// Builds the trees of one family (build_tree, module_localization.f90:35-167) and their
// column tables.  Appends TreeDesc entries.
int build_family(int family, const cwbl_var_params *vp, std::vector<TreeDesc> &descs,
                 int &list_cap, int &max_depth) {
  struct Pending { int entry; int type_id; const cwbl_type_params *tp; float hinv, vinv; };
  std::vector<Pending> pend;
  const int ntypes = family == 0 ? CWBL_NUM_GTS_TYPES : CWBL_NUM_RADAR_TYPES;
  for (int id = 1; id <= ntypes; ++id) {
    int entry = -1;
    for (size_t e = 0; e < S.obs.size(); ++e)
      if (S.obs[e].family == family && S.obs[e].type_id == id) entry = (int)e;
    if (entry < 0 || S.obs[entry].nobs <= 0) continue;
    if (family == 0 && !is_gts_assimilated(id)) continue;
    const cwbl_type_params *tp = family == 0 ? &vp->gts[id - 1] : &vp->radar[id - 1];
    if (!(tp->use_it && tp->hclr > 0.0f)) continue;
    if (tp->max_lz_pts < 0) return fail(CWBL_ERR_ARG, "max_lz_pts < 0 for type %d", id);
    const float hinv = 1.0f / (tp->hclr * 1e3f);
    const float vinv = tp->vclr > 0.0f ? 1.0f / (tp->vclr * 1e3f) : -1.0f;
    pend.push_back({entry, id, tp, hinv, vinv});
  }
  if (pend.empty()) return CWBL_OK;
  const bool fam3d = pend.back().vinv > 0.0f;  // Q1: the leftover vclr_inv (:151)
  for (const Pending &pd : pend) {
    ObsType &ot = S.obs[pd.entry];
    const bool own3d = pd.vinv > 0.0f;
    bool dim3 = S.q1_mode == CWBL_Q1_PER_TYPE ? own3d : fam3d;
    int q1u = 0;
    if (dim3 && !own3d) { dim3 = false; q1u = 1; }
    const int n = ot.nobs;
    const int tdim = dim3 ? 3 : 2;
    TreeBufs *tb = nullptr;
    for (auto &t : S.tree_cache)
      if (t->entry == pd.entry && t->dim == tdim && t->hinv == pd.hinv &&
          (!dim3 || t->vinv == pd.vinv) && t->bin_div_opt == S.bin_div)
        tb = t.get();
    if (!tb) {  // build_tree (:35-167) for this normalisation
      std::vector<float> nx(3 * (size_t)n);
      for (int j = 0; j < n; ++j) {
        nx[3 * j + 0] = ot.xyz[3 * j + 0] * pd.hinv;
        nx[3 * j + 1] = ot.xyz[3 * j + 1] * pd.hinv;
        nx[3 * j + 2] = dim3 ? ot.xyz[3 * j + 2] * pd.vinv : -1.0f;
      }
      auto nt = std::make_unique<TreeBufs>();
      nt->entry = pd.entry; nt->dim = tdim; nt->hinv = pd.hinv; nt->vinv = pd.vinv;
      nt->bin_div_opt = S.bin_div;
      build_kdtree(nx.data(), n, tdim, nt->host);
      nt->depth = tree_depth(nt->host);
      if (nt->depth >= kSearchStackDepth)
        return fail(CWBL_ERR_UNSUPPORTED, "k-d tree too deep (%d obs)", n);
      const HostTree &h = nt->host;
      HIPCHK(nt->nodes.ensure(h.nodes.size() * sizeof(TreeNode)));
      HIPCHK(nt->rdata.ensure(h.rdata.size() * sizeof(float)));
      HIPCHK(nt->ind.ensure(h.ind.size() * sizeof(int) + 4));
      HIPCHK(hipMemcpyAsync(nt->nodes.p, h.nodes.data(), h.nodes.size() * sizeof(TreeNode),
                            hipMemcpyHostToDevice, S.stream));
      HIPCHK(hipMemcpyAsync(nt->rdata.p, h.rdata.data(), h.rdata.size() * sizeof(float),
                            hipMemcpyHostToDevice, S.stream));
      if (!h.ind.empty())
        HIPCHK(hipMemcpyAsync(nt->ind.p, h.ind.data(), h.ind.size() * sizeof(int),
                              hipMemcpyHostToDevice, S.stream));
      build_bins(h, tdim, std::sqrt(search_r2()), nt->bins, bin_div_for(h, tdim));
      const HostBins &hb = nt->bins;
      // (+ kBinPad points: search_binned_kernel reads up to 7 points past a run's end)
      HIPCHK(nt->bxyz.ensure(hb.xyzs.size() * sizeof(float) + 16 * kBinPad));
      HIPCHK(nt->bstart.ensure(hb.start.size() * sizeof(int)));
      if (!hb.xyzs.empty())
        HIPCHK(hipMemcpyAsync(nt->bxyz.p, hb.xyzs.data(), hb.xyzs.size() * sizeof(float),
                              hipMemcpyHostToDevice, S.stream));
      HIPCHK(hipMemcpyAsync(nt->bstart.p, hb.start.data(), hb.start.size() * sizeof(int),
                            hipMemcpyHostToDevice, S.stream));
      tb = nt.get();
      S.tree_cache.push_back(std::move(nt));
    }
    const size_t ncol = (size_t)n * ot.nvar;
    HIPCHK(tb->col_bg.ensure(ncol * S.kp * sizeof(float)));
    HIPCHK(tb->col_omm.ensure(ncol * sizeof(float)));
    HIPCHK(tb->col_err.ensure(ncol * sizeof(float)));
    HIPCHK(tb->col_ok.ensure(ncol));
    // point-independent QC columns (letkf_yoyb :429-437 / :497-510)
    const cwbl_type_params *tp = pd.tp;
    int is_assim[5] = {0, 0, 0, 0, 0};
    if (family == 0) {
      for (int v = 0; v < ot.nvar; ++v) is_assim[v] = tp->hclr > 0.0f ? tp->is_assim[v] : 0;
    } else {
      is_assim[0] = tp->hclr > 0.0f ? 1 : 0;
    }
    HIPCHK(launch_obs_prep(S.stream, S.k, S.kp, family, ot.type_id, ot.nvar, n,
                           ot.obs.as<float>(), ot.error.as<float>(), ot.hdxb.as<float>(),
                           ot.qc.as<int>(), tp->err_muti, tp->err_rej, is_assim, S.norain,
                           tb->ind.as<int>(), tb->col_bg.as<float>(), tb->col_omm.as<float>(),
                           tb->col_err.as<float>(), tb->col_ok.as<uint8_t>()));
    TreeDesc d{};
    d.nodes = tb->nodes.as<TreeNode>();
    d.rdata = tb->rdata.as<float4>();
    d.ind = tb->ind.as<int>();
    d.col_bg = tb->col_bg.as<float>();
    d.col_omm = tb->col_omm.as<float>();
    d.col_err = tb->col_err.as<float>();
    d.col_ok = tb->col_ok.as<uint8_t>();
    d.hclr_inv = pd.hinv;
    d.vclr_inv = pd.vinv;
    d.tree_dim = dim3 ? 3 : 2;
    d.query3d = own3d ? 1 : 0;
    d.nvar = ot.nvar;
    d.max_lz = tp->max_lz_pts;
    d.list_off = list_cap;
    d.q1_undef = q1u;
    d.bxyz = tb->bxyz.as<float4>();
    d.bstart = tb->bstart.as<int>();
    d.bx0 = tb->bins.x0; d.by0 = tb->bins.y0; d.bz0 = tb->bins.z0; d.binv = tb->bins.binv;
    d.nbx = tb->bins.nbx; d.nby = tb->bins.nby; d.nbz = tb->bins.nbz;
    list_cap += list_span(tp->max_lz_pts);
    max_depth = std::max(max_depth, tb->depth);
    descs.push_back(d);
  }
  return CWBL_OK;
}

void release_obs() {
  for (auto &t : S.tree_cache) t->release();
  S.tree_cache.clear();
  for (auto &o : S.obs) {
    o.obs.release(); o.error.release(); o.hdxb.release(); o.qc.release();
  }
  S.obs.clear();
  S.have_obs = false;
}

void release_all() {
  release_obs();
  for (hipEvent_t e : S.cevents) (void)hipEventDestroy(e);
  S.cevents.clear();
  for (DevBuf *b : {&S.tdesc, &S.nbr_cnt, &S.nbr_idx, &S.nbr_cnt2, &S.nbr_idx2, &S.info, &S.stats, &S.sx,
                    &S.sy, &S.salt, &S.svar, &S.bcol, &S.byo, &S.byb, &S.bxb, &S.bxa, &S.bev, &S.btri,
                    &S.qxyz, &S.qnf, &S.qidx, &S.qr2, &S.quad, &S.wsa, &S.flags})
    b->release();
  for (hipEvent_t e : S.events) (void)hipEventDestroy(e);
  S.events.clear();
  for (hipEvent_t e : S.kevents) (void)hipEventDestroy(e);
  S.kevents.clear();
  for (int i = 0; i < State::kSlots; ++i) {
    S.pin_in[i].release();
    S.pin_out[i].release();
  }
  S.pool.stop();
  S.kpend.clear();
  S.kev_used = 0;
  S.ktiming = false;
  for (KTime &t : S.ktime) t = KTime{};
  if (S.order_ev) (void)hipEventDestroy(S.order_ev);
  S.order_ev = nullptr;
  S.caller_stream = nullptr;
  if (S.stream) (void)hipStreamDestroy(S.stream);
  S.stream = nullptr;
  if (S.sstream) (void)hipStreamDestroy(S.sstream);
  S.sstream = nullptr;
  for (hipStream_t *st : {&S.h2d, &S.d2h}) {
    if (*st) (void)hipStreamDestroy(*st);
    *st = nullptr;
  }
  S.inited = false;
}

// k = 17..32: the KP = 40 record path (assembly + four-point solve; the padding rows are
// the identity and the steps past k - 2 exact no-ops) beats the one-wavefront KP = 24 / 32
// solves (C2 grid, r2: 91.6 against 134 ms per variable at k = 32; r3: ~75 against 79 / 88
// at k = 20 / 24); at k <= 16 the one-wavefront solve is faster (68 ms)
void select_kp() {
  S.kp = S.kp_natural;
  if ((S.kp == 24 || S.kp == 32) && S.tq4 && !S.jacobi) S.kp = kTq4KP;
}

SolveConsts solve_consts(float inflat, int use_rtpp, float rtpp_a, int use_rtps, float rtps_a) {
  SolveConsts c{};
  c.k = S.k;
  c.kp = S.kp;
  c.weight_function = S.wf;
  c.inflat = inflat;
  c.use_rtpp = use_rtpp;
  c.use_rtps = use_rtps;
  c.rtpp_alpha = rtpp_a;
  c.rtps_alpha = rtps_a;
  c.nmember_inv = 1.0f / (float)S.k;
  c.r2 = search_r2();
  c.max_sweeps = 30;
  c.quad_r = S.quad.as<double2>();
  c.quad = c.quad_r;
#ifdef CWBL_DEBUG_KNOBS  // timing ablations (make DEBUG_KNOBS=1); not in the release library
  if (const char *e = std::getenv("CWBL_DEBUG_MAX_SWEEPS")) c.max_sweeps = std::atoi(e);
  if (const char *e = std::getenv("CWBL_DEBUG_TQ_STOP")) c.debug_stop = std::atoi(e);
  if (const char *e = std::getenv("CWBL_DEBUG_TQ_STEPS")) c.debug_steps = std::atoi(e);
#endif
  return c;
}

// ---- cwbl_analyze_var by stage ---------------------------------------------------------------
// One call of cwbl_analyze_var (letkf_driver's per-variable body, module_letkf_core.f90:59-297):
//   plan_trees      build_tree x2 (cached per obs set) + the QC column tables   (:63-64)
//   stage_slab      the slab in device memory (host slabs staged / piped)
//   plan_batches    search/solve batches
//   per batch       search_batch (S.sstream) -> solve_batch_path (S.stream), with the host
//                   slab's var piped in and out around it (S.h2d / S.d2h)        (:209-240)
//   finish_call     info reduction, tune_q (:253-278), write-back, statistics
struct VarCall {
  const cwbl_var_params *vp = nullptr;
  const cwbl_slab *sl = nullptr;
  long long npts = 0, L = 0;
  SlabDev sd{};
  size_t bvar = 0;
  // host-memory slab: x, y, alt staged first; var piped batch by batch (piped: the analysed
  // region is the whole horizontal slab, so a batch's points are contiguous in every member
  // plane) or moved whole; a pageable var page-locked in place (registered) or, failing that,
  // through the library's page-locked bounce slots
  bool host = false, piped = false, piped_back = false, bounce = false, registered = false;
  std::vector<TreeDesc> descs;
  int list_cap = 0, max_depth = 1, nt = 0;
  std::vector<std::pair<long long, int>> plan;  // (g0, nb)
  long long B = 0, Bc = 0, info_cap = 0, win0 = 0;
  SolveConsts c{};
  float rbox = 0.0f;
  // timing events S.events[ev..] (four per batch: search begin/end, solve begin/end) and
  // ordering events S.cevents[cev..] of the piped copies
  int ev = 4, cev = 0;
  std::vector<std::pair<int, int>> search_ev, solve_ev;
  std::vector<int> done_ev, h2d_done, d2h_done;
};

// build_tree of both families and the upload of their descriptors (nt = 0: nothing to do)
int plan_trees(VarCall &v) {
  if (int rc = build_family(0, v.vp, v.descs, v.list_cap, v.max_depth)) return rc;
  if (int rc = build_family(1, v.vp, v.descs, v.list_cap, v.max_depth)) return rc;
  v.nt = (int)v.descs.size();
  if (v.nt == 0 || v.npts == 0) return CWBL_OK;
  HIPCHK(S.tdesc.ensure(v.descs.size() * sizeof(TreeDesc)));
  HIPCHK(hipMemcpyAsync(S.tdesc.p, v.descs.data(), v.descs.size() * sizeof(TreeDesc),
                        hipMemcpyHostToDevice, S.stream));
  return CWBL_OK;
}

int stage_slab(VarCall &v) {
  const cwbl_slab *sl = v.sl;
  v.L = (long long)sl->nx * sl->ny * sl->nz;
  SlabDev &sd = v.sd;
  sd.nx = sl->nx; sd.ny = sl->ny; sd.nz = sl->nz; sd.alt_nx = sl->alt_nx;
  sd.alt_ny = sl->alt_ny; sd.ix_lim = sl->ix_lim; sd.iy_lim = sl->iy_lim; sd.L = v.L;
  const size_t bxy = (size_t)sl->nx * sl->ny * 4;
  const size_t balt = (size_t)sl->alt_nx * sl->alt_ny * sl->nz * 4;
  v.bvar = (size_t)v.L * S.k * 4;
  v.host = sl->memory != CWBL_MEM_DEVICE;
  v.piped = v.host && sl->ix_lim == sl->nx && sl->iy_lim == sl->ny;
  v.piped_back = v.piped && !v.vp->tune_q;  // tune_q touches the whole slab afterwards
  // pageable var (a Fortran host's ordinary arrays): copies from pageable memory are staged by
  // the runtime and do not overlap.  It is page-locked in place for the call (r4, C2 from
  // pageable numpy arrays: 58.7 M pts/s, against 58.2 M page-locked and 50.8 M through the
  // bounce slots, whose host copies stall the pipeline); the slots remain the fallback when
  // the registration fails (and CWBL_OPT_PAGEABLE = 1 forces them)
  v.bounce = v.host && v.bvar > 0 && !host_pinned(sl->var);
  if (v.bounce && S.pageable_register) {
    if (hipHostRegister(sl->var, v.bvar, hipHostRegisterDefault) == hipSuccess) {
      v.registered = true;
      v.bounce = false;
    } else {
      (void)hipGetLastError();
    }
  }
  if (!v.host) {
    sd.x = sl->x; sd.y = sl->y; sd.alt = sl->alt; sd.var = sl->var;
    return CWBL_OK;
  }
  HIPCHK(stage(S.sx, sl->x, bxy, CWBL_MEM_HOST));
  HIPCHK(stage(S.sy, sl->y, bxy, CWBL_MEM_HOST));
  HIPCHK(stage(S.salt, sl->alt, balt, CWBL_MEM_HOST));
  if (v.piped || v.bounce) HIPCHK(S.svar.ensure(v.bvar));
  else HIPCHK(stage(S.svar, sl->var, v.bvar, CWBL_MEM_HOST));
  sd.x = S.sx.as<float>(); sd.y = S.sy.as<float>(); sd.alt = S.salt.as<float>();
  sd.var = S.svar.as<float>();
  return CWBL_OK;
}

void plan_batches(VarCall &v) {
  const long long npts = v.npts;
  const size_t per_pt = (size_t)v.list_cap * 4 + (size_t)v.nt * 4 + 8;
  long long B = (long long)(S.ws_bytes / per_pt);
  B = std::min<long long>(B, S.max_batch);
  // at least ~6 batches while they stay above 64 k points: with few batches the first search
  // and the last solve run alone (an 8-GPU rank's C2 share, 562 k points: 12.8 ms per step
  // in batches of 141 k, 12.3 in batches of 94 k; the full grid is indifferent in 100-160 k)
  if (!S.max_batch_set) B = std::min<long long>(B, std::max<long long>(npts / 6, 64000));
  B = std::max<long long>(std::min<long long>(B, npts), 256);
  B = std::min<long long>(B, 1 << 22);
  // a batch's lists stay below 4 GiB: search_binned_kernel addresses them by 32-bit offsets
  if (v.list_cap > 0)
    B = std::min<long long>(B, (long long)((((size_t)1 << 32) - 1) / ((size_t)v.list_cap * 4)) /
                                   kListLanes * kListLanes);
  // The first batch's search cannot overlap a solve, so it may be short (a lead of
  // 1/lead_div of the points); the rest are equal (a short last batch is all tail) and whole
  // list groups.
  const auto round_up = [](long long x) { return (x + kListLanes - 1) / kListLanes * kListLanes; };
  long long lead = S.lead_div > 0 ? round_up(npts / S.lead_div) : 0;
  if (lead < 4 * kListLanes || lead >= npts) lead = 0;
  if (lead > 0) v.plan.push_back({0, (int)std::min<long long>(lead, B)});
  const long long g1 = v.plan.empty() ? 0 : v.plan[0].second, rest = npts - g1;
  const long long nrest = (rest + B - 1) / B;
  const long long Br = round_up((rest + nrest - 1) / nrest);
  for (long long g = g1; g < npts; g += Br)
    v.plan.push_back({g, (int)std::min<long long>(Br, npts - g)});
  v.B = 0;
  for (const auto &b : v.plan) v.B = std::max<long long>(v.B, b.second);
  // bounce slots: one batch (or one whole-slab chunk of Bc points) of k member rows each
  v.Bc = std::min<long long>(std::max<long long>(v.B, 1), std::max<long long>(v.L, 1));
  // the per-point info of a window of up to S.info_window points is reduced once per window
  // (a reduction kernel per batch cost the C2 step ~0.5 ms)
  v.info_cap = std::max<long long>(v.B, std::min<long long>(npts, S.info_window));
}

// Whole-slab moves through the bounce slots (var not piped, or back after tune_q): chunk i of
// Bc points of every member row.  Up: fill slot i & 1 (once its copy two chunks back has left
// it), copy up on S.stream.  Down: copy chunk i down on S.stream, drain chunk i - 1 meanwhile.
int bounce_whole(VarCall &v, bool up) {
  std::vector<int> evs;
  long long pc0 = 0;
  int pcn = 0;
  const size_t pitch = (size_t)v.L * 4;
  float *const hvar = v.sl->var;
  for (long long c0 = 0, i = 0; c0 < v.L; c0 += v.Bc, ++i) {
    const int cn = (int)std::min<long long>(v.Bc, v.L - c0);
    PinBuf &slot = up ? S.pin_in[i & 1] : S.pin_out[i & 1];
    hipEvent_t e;
    HIPCHK(cevent(v.cev, &e));
    if (up) {
      if (i >= 2) HIPCHK(hipEventSynchronize(S.cevents[evs[(size_t)i - 2]]));
      bounce_rows(S.pool, slot.as<float>(), hvar, v.L, c0, cn, S.k, true);
      HIPCHK(hipMemcpy2DAsync(S.svar.as<float>() + c0, pitch, slot.p, (size_t)cn * 4,
                              (size_t)cn * 4, (size_t)S.k, hipMemcpyHostToDevice, S.stream));
    } else {
      HIPCHK(hipMemcpy2DAsync(slot.p, (size_t)cn * 4, S.svar.as<float>() + c0, pitch,
                              (size_t)cn * 4, (size_t)S.k, hipMemcpyDeviceToHost, S.stream));
    }
    HIPCHK(hipEventRecord(e, S.stream));
    evs.push_back(v.cev++);
    if (!up && i >= 1) {
      HIPCHK(hipEventSynchronize(S.cevents[evs[(size_t)i - 1]]));
      bounce_rows(S.pool, S.pin_out[(i - 1) & 1].as<float>(), hvar, v.L, pc0, pcn, S.k, false);
    }
    pc0 = c0;
    pcn = cn;
  }
  if (!up && !evs.empty()) {
    HIPCHK(hipEventSynchronize(S.cevents[evs.back()]));
    bounce_rows(S.pool, S.pin_out[(evs.size() - 1) & 1].as<float>(), hvar, v.L, pc0, pcn,
                S.k, false);
  }
  return CWBL_OK;
}

// Piped bounce: batch b's columns into slot b % kSlots once the copy up of batch b - kSlots
// has left it; batch b's analysis out of its slot once its copy down is done.
int bounce_fill(VarCall &v, long long b) {
  if (b >= State::kSlots) HIPCHK(hipEventSynchronize(S.cevents[v.h2d_done[b - State::kSlots]]));
  bounce_rows(S.pool, S.pin_in[b % State::kSlots].as<float>(), v.sl->var, v.L, v.plan[b].first,
              v.plan[b].second, S.k, true);
  return CWBL_OK;
}

int bounce_drain(VarCall &v, long long b) {
  HIPCHK(hipEventSynchronize(S.cevents[v.d2h_done[b]]));
  bounce_rows(S.pool, S.pin_out[b % State::kSlots].as<float>(), v.sl->var, v.L, v.plan[b].first,
              v.plan[b].second, S.k, false);
  return CWBL_OK;
}

// The bounce slots of this call (page-locked only while a call needs them) and the whole-slab
// move up when var is not piped.
int stage_bounce(VarCall &v) {
  if (v.registered) {  // the slots are only the fallback's: give them back
    for (int i = 0; i < State::kSlots; ++i) {
      S.pin_in[i].release();
      S.pin_out[i].release();
    }
  }
  if (!v.bounce) return CWBL_OK;
  const size_t slot_bytes = (size_t)v.Bc * S.k * 4;
  const int nin = v.piped ? State::kSlots : 2, nout = v.piped_back ? State::kSlots : 2;
  for (int i = 0; i < nin; ++i) HIPCHK(S.pin_in[i].ensure(slot_bytes));
  for (int i = 0; i < nout; ++i) HIPCHK(S.pin_out[i].ensure(slot_bytes));
  if (!v.piped) return bounce_whole(v, true);
  return CWBL_OK;
}

// Per-call device buffers (two neighbour-list buffers: the search of batch b + 1 overlaps the
// solve of batch b) and the solve constants.
int alloc_call_buffers(VarCall &v) {
  const long long B = v.B;
  const size_t bytes_cnt = (size_t)B * v.nt * 4;
  const size_t bytes_idx =
      (size_t)((B + kListLanes - 1) / kListLanes) * kListLanes * std::max(v.list_cap, 1) * 4;
  HIPCHK(S.nbr_cnt.ensure(bytes_cnt));
  HIPCHK(S.nbr_idx.ensure(bytes_idx));
  if (v.plan.size() > 1) {
    HIPCHK(S.nbr_cnt2.ensure(bytes_cnt));
    HIPCHK(S.nbr_idx2.ensure(bytes_idx));
  }
  HIPCHK(S.flags.ensure((size_t)(B + 1) * sizeof(int)));
  HIPCHK(S.stats.ensure(sizeof(DevStats)));
  HIPCHK(hipMemsetAsync(S.stats.p, 0, sizeof(DevStats), S.stream));
  HIPCHK(S.info.ensure((size_t)v.info_cap * sizeof(int2)));
  v.c = solve_consts((float)(S.k - 1) / v.vp->multi_infl,  // inflat (:68)
                     v.vp->use_rtpp, v.vp->rtpp_alpha, v.vp->use_rtps, v.vp->rtps_alpha);
  v.c.ntrees = v.nt;
  v.c.list_cap = v.list_cap;
  // bounding-box half-width of the binned search: the radius with a margin, so that every
  // point with d2 <= r2 in fp32 lies inside
  v.rbox = std::sqrt(search_r2()) * 1.0001f + 1e-5f;
  return CWBL_OK;
}

// get_lz for every point of batch bi (module_localization.f90:188-331) on S.sstream: uniform
// bins, then the k-d tree walk for the points whose lists pass max_lz_pts (Q4); or the tree
// walk for every point (CWBL_OPT_SEARCH = 1).  Waits for the solve two batches back, which
// read the same list buffer.
int search_batch(VarCall &v, long long bi, int *ncnt, int *nidx, hipEvent_t a, hipEvent_t b) {
  const long long g0 = v.plan[bi].first;
  const int nb = v.plan[bi].second;
  const TreeDesc *dtrees = S.tdesc.as<TreeDesc>();
  DevStats *dst = S.stats.as<DevStats>();
  // (timing experiment: CWBL_DEBUG_SERIAL=1 runs the searches on the solve stream)
  hipStream_t ss = S.serial_search ? S.stream : S.sstream;
  if (bi >= 2) HIPCHK(hipStreamWaitEvent(ss, S.events[v.done_ev[bi - 2]], 0));
  HIPCHK(hipEventRecord(a, ss));
  int kt;
  if (S.binned) {
    int *fcnt = S.flags.as<int>(), *fidx = fcnt + 1;
    HIPCHK(hipMemsetAsync(fcnt, 0, sizeof(int), ss));
    HIPCHK(kt_begin(ss, &kt));
    HIPCHK(launch_search_binned(ss, dtrees, v.nt, v.list_cap, v.c.r2, v.rbox, v.sd, g0, nb, ncnt,
                                nidx, fcnt, fidx));
    HIPCHK(kt_end(ss, kt, KT_SEARCH_BINNED, nb));
    HIPCHK(kt_begin(ss, &kt));
    HIPCHK(launch_search_flagged(ss, dtrees, v.nt, v.max_depth, v.list_cap, v.c.r2, v.sd, g0, nb,
                                 fcnt, fidx, ncnt, nidx, dst));
    HIPCHK(kt_end(ss, kt, KT_SEARCH_FLAGGED, 0));
  } else {
    HIPCHK(kt_begin(ss, &kt));
    HIPCHK(launch_search(ss, dtrees, v.nt, v.max_depth, v.list_cap, v.c.r2, v.sd, g0, nb, ncnt,
                         nidx, nullptr, dst));
    HIPCHK(kt_end(ss, kt, KT_SEARCH_TREE, nb));
  }
  return hipEventRecord(b, ss) == hipSuccess ? CWBL_OK
                                              : fail(CWBL_ERR_HIP, "search event record failed");
}

// A host slab's var columns of batch bi up (k rows of nb floats, member pitch L) on S.h2d,
// from the caller's page-locked array or from the batch's bounce slot; S.stream waits.
int upload_batch_var(VarCall &v, long long bi) {
  const long long g0 = v.plan[bi].first;
  const int nb = v.plan[bi].second;
  hipEvent_t hv;
  const int hv_i = v.cev++;
  HIPCHK(cevent(hv_i, &hv));
  const size_t pitch = (size_t)v.L * 4;
  if (v.bounce) {  // slot bi % kSlots, filled before this batch (bounce_fill)
    if (bi == 0)
      if (int rc = bounce_fill(v, 0)) return rc;
    HIPCHK(hipMemcpy2DAsync(S.svar.as<float>() + g0, pitch, S.pin_in[bi % State::kSlots].p,
                            (size_t)nb * 4, (size_t)nb * 4, (size_t)S.k, hipMemcpyHostToDevice,
                            S.h2d));
  } else {
    HIPCHK(hipMemcpy2DAsync(S.svar.as<float>() + g0, pitch, v.sl->var + g0, pitch,
                            (size_t)nb * 4, (size_t)S.k, hipMemcpyHostToDevice, S.h2d));
  }
  HIPCHK(hipEventRecord(hv, S.h2d));
  v.h2d_done.push_back(hv_i);
  HIPCHK(hipStreamWaitEvent(S.stream, hv, 0));
  return CWBL_OK;
}

// Batch bi's analysis back to a host slab behind its solve (event dn) on S.d2h.
int return_batch_var(VarCall &v, long long bi, hipEvent_t dn) {
  const long long g0 = v.plan[bi].first;
  const int nb = v.plan[bi].second;
  HIPCHK(hipStreamWaitEvent(S.d2h, dn, 0));
  const size_t pitch = (size_t)v.L * 4;
  if (v.bounce) {  // into slot bi % kSlots (drained kSlots - 1 batches later)
    hipEvent_t dv;
    const int dv_i = v.cev++;
    HIPCHK(cevent(dv_i, &dv));
    HIPCHK(hipMemcpy2DAsync(S.pin_out[bi % State::kSlots].p, (size_t)nb * 4,
                            S.svar.as<float>() + g0, pitch, (size_t)nb * 4, (size_t)S.k,
                            hipMemcpyDeviceToHost, S.d2h));
    HIPCHK(hipEventRecord(dv, S.d2h));
    v.d2h_done.push_back(dv_i);
  } else {
    HIPCHK(hipMemcpy2DAsync(v.sl->var + g0, pitch, S.svar.as<float>() + g0, pitch,
                            (size_t)nb * 4, (size_t)S.k, hipMemcpyDeviceToHost, S.d2h));
  }
  return CWBL_OK;
}

// Sub-batches of a search batch for a path with a per-point record: ns points (a multiple of
// kListLanes, so a sub-batch's neighbour lists start on a list group) with at most `cap`
// points each, the batch split evenly.
long long sub_batch(int nb, long long cap) {
  const long long nsub = (nb + cap - 1) / cap;
  const long long Bs = (nb + nsub - 1) / nsub;
  return std::max<long long>(kListLanes, (Bs + kListLanes - 1) / kListLanes * kListLanes);
}

// letkf_yoyb + letkf_solve (module_letkf_core.f90:300-700) for batch (g0, nb) on S.stream, one
// path per ensemble-size class:
//   k = 17..40   record path: assemble_record_kernel -> record -> solve_tq40_kernel
//   k = 65..128  hand-off path: 256-thread kernel (assembly + first steps) -> record ->
//                solve_tqb_tail_kernel; CWBL_OPT_BIG_PATH = 0: one 256-thread kernel
//   otherwise    one wavefront per point: solve_tq_kernel; CWBL_OPT_SOLVER = 1: the Jacobi
//                eigensolver kernel (k <= 64)
// b2 / dn: the events around the batch's solve (the record path times its kernel pair
// between them).
int solve_batch_path(VarCall &v, long long g0, int nb, const int *ncnt, const int *nidx,
                     int2 *infob, hipEvent_t b2, hipEvent_t dn) {
  const TreeDesc *dtrees = S.tdesc.as<TreeDesc>();
  const SolveConsts &c = v.c;
  const SlabDev &sd = v.sd;
  const int nt = v.nt, list_cap = v.list_cap;
  int kt;
  const bool handoff = (S.kp == 96 || S.kp == kBigSplitKP) && S.big_split &&
                       S.k > big_split_j0(S.kp) + 2;
  if (S.tq4 && S.kp == kTq4KP && !S.jacobi) {
    // (Bs <= 2^19: the solve addresses a sub-batch's records with 32-bit byte offsets)
    const long long cap = std::min<long long>(S.tq4_sub > 0 ? S.tq4_sub : nb, 1 << 19);
    const long long Bs = std::min<long long>(sub_batch(nb, cap), 1 << 19);
    // (+1: the spare record of solve_tq40_kernel's lanes past the sub-batch)
    HIPCHK(S.wsa.ensure((size_t)(Bs + 1) * 8 * AsmRecord<kTq4KP>::WORDS));
    double *rec = S.wsa.as<double>();
    if (Bs >= nb) {  // the whole batch: timed between b2 and dn (recorded anyway)
      auto asm_ = [&]() {
        return launch_assemble_record(S.stream, S.kp, dtrees, c, sd, g0, nb, ncnt, nidx, infob,
                                      rec);
      };
      auto tq40 = [&]() { return launch_solve_tq40(S.stream, S.kp, c, sd, g0, nb, rec, infob); };
      HIPCHK(kt_pair(S.stream, b2, KT_ASSEMBLE_RECORD, nb, dn, KT_SOLVE_TQ40, nb, asm_, tq40));
      return CWBL_OK;
    }
    for (long long s0 = 0; s0 < nb; s0 += Bs) {
      const int ns = (int)std::min<long long>(Bs, nb - s0);
      HIPCHK(kt_begin(S.stream, &kt));
      HIPCHK(launch_assemble_record(S.stream, S.kp, dtrees, c, sd, g0 + s0, ns, ncnt + s0 * nt,
                                    nidx + s0 * list_cap, infob + s0, rec));
      HIPCHK(kt_end(S.stream, kt, KT_ASSEMBLE_RECORD, ns));
      HIPCHK(kt_begin(S.stream, &kt));
      HIPCHK(launch_solve_tq40(S.stream, S.kp, c, sd, g0 + s0, ns, rec, infob + s0));
      HIPCHK(kt_end(S.stream, kt, KT_SOLVE_TQ40, ns));
    }
    return CWBL_OK;
  }
  if (handoff) {
    // BigHandoff<128, 64> is 134.7 KB per point (13 GB at the default 98 304-point
    // sub-batch, outside workspace_bytes); the sub-batch is also bounded by the hand-off
    // budget (cwbl_init: workspace_bytes when the caller gave one, else 13 GB or 40% of the
    // free device memory)
    const size_t rec_bytes = (size_t)8 * (S.kp == 96 ? BigHandoff<96, 32>::WORDS
                                                     : BigHandoff<kBigSplitKP, kBigJ0>::WORDS);
    const long long fit = std::max<long long>(
        kListLanes, (long long)(S.handoff_budget / rec_bytes) / kListLanes * kListLanes);
    const long long Bs = sub_batch(nb, std::min<long long>(S.big_sub, fit));
    HIPCHK(S.wsa.ensure((size_t)Bs * rec_bytes));
    for (long long s0 = 0; s0 < nb; s0 += Bs) {
      const int ns = (int)std::min<long long>(Bs, nb - s0);
      HIPCHK(kt_begin(S.stream, &kt));
      HIPCHK(launch_big_handoff(S.stream, S.kp, dtrees, c, sd, g0 + s0, ns, ncnt + s0 * nt,
                                nidx + s0 * list_cap, infob + s0, S.wsa.as<double>()));
      HIPCHK(kt_end(S.stream, kt, KT_BIG_HANDOFF, ns));
      HIPCHK(kt_begin(S.stream, &kt));
      HIPCHK(launch_solve_tqb_tail(S.stream, S.kp, c, sd, g0 + s0, ns, S.wsa.as<double>(),
                                   infob + s0));
      HIPCHK(kt_end(S.stream, kt, KT_TQB_TAIL, ns));
    }
    return CWBL_OK;
  }
  HIPCHK(kt_begin(S.stream, &kt));
  if (S.kp > kMaxWaveKP) {
    HIPCHK(launch_solve_tq_big(S.stream, S.kp, false, dtrees, c, sd, g0, nb, ncnt, nidx,
                               nullptr, nullptr, nullptr, nullptr, nullptr, infob));
    HIPCHK(kt_end(S.stream, kt, KT_SOLVE_TQ_BIG, nb));
  } else if (S.jacobi) {
    HIPCHK(launch_solve_neighbors(S.stream, S.kp, dtrees, c, sd, g0, nb, ncnt, nidx, infob));
    HIPCHK(kt_end(S.stream, kt, KT_SOLVE_JACOBI, nb));
  } else {
    HIPCHK(launch_solve_tq(S.stream, S.kp, false, dtrees, c, sd, g0, nb, ncnt, nidx, nullptr,
                           nullptr, nullptr, nullptr, nullptr, infob));
    HIPCHK(kt_end(S.stream, kt, KT_SOLVE_TQ, nb));
  }
  return CWBL_OK;
}

// After the last batch: the info of the open window, tune_q on the resident slab
// (letkf_driver's Q species post-step, :253-278), the host slab's var back, one
// synchronisation, and the statistics.
int finish_call(VarCall &v, cwbl_stats &st) {
  DevStats *dst = S.stats.as<DevStats>();
  if (v.npts > v.win0)
    HIPCHK(launch_reduce_info(S.stream, S.info.as<int2>(), (int)(v.npts - v.win0), dst));
  int ev = v.ev;
  if (v.vp->tune_q) {
    hipEvent_t a, b;
    HIPCHK(event(ev, &a));
    HIPCHK(event(ev + 1, &b));
    HIPCHK(hipEventRecord(a, S.stream));
    int kt;
    HIPCHK(kt_begin(S.stream, &kt));
    HIPCHK(launch_tune_q(S.stream, v.sd, S.k));
    HIPCHK(kt_end(S.stream, kt, KT_TUNE_Q, v.npts));
    HIPCHK(hipEventRecord(b, S.stream));
    v.solve_ev.push_back({ev, ev + 1});
    ev += 2;
  }
  hipEvent_t e_end, e_back;
  HIPCHK(event(ev, &e_end));
  HIPCHK(event(ev + 1, &e_back));
  if (v.host && !v.piped_back && !v.bounce)
    HIPCHK(hipMemcpyAsync(v.sl->var, S.svar.p, v.bvar, hipMemcpyDeviceToHost, S.stream));
  if (v.piped_back) {  // the call returns after the last batch's copy back
    HIPCHK(hipEventRecord(e_back, S.d2h));
    HIPCHK(hipStreamWaitEvent(S.stream, e_back, 0));
  }
  const long long nbat = (long long)v.plan.size();
  if (v.bounce && v.piped_back)  // drain the last batches
    for (long long bj = std::max<long long>(0, nbat - (State::kSlots - 1)); bj < nbat; ++bj)
      if (int rc = bounce_drain(v, bj)) return rc;
  if (v.bounce && !v.piped_back)  // the whole slab back (after tune_q, or a staggered slab)
    if (int rc = bounce_whole(v, false)) return rc;
  HIPCHK(hipEventRecord(e_end, S.stream));
  DevStats ds;
  HIPCHK(hipMemcpyAsync(&ds, S.stats.p, sizeof ds, hipMemcpyDeviceToHost, S.stream));
  HIPCHK(hipStreamSynchronize(S.stream));
  kt_collect();

  st.solved = (long long)ds.solved;
  st.nobs_sum = (long long)ds.nobs_sum;
  st.lz_truncated = (long long)ds.lz_truncated;
  st.nonconverged = (long long)ds.nonconverged;
  st.sweeps_sum = (long long)ds.sweeps_sum;
  st.max_p = (int)ds.max_p;
  st.max_sweeps = (int)ds.max_sweeps;
  st.ms_prep = elapsed(0, 1);
  for (auto &p : v.search_ev) st.ms_search += elapsed(p.first, p.second);
  for (auto &p : v.solve_ev) st.ms_solve += elapsed(p.first, p.second);
  // copies: x, y, alt (+ var when not piped) before the batches, var back after the last
  // solve; piped transfers overlap the batches and are not counted here
  st.ms_copy = elapsed(1, 2) + (v.host && !v.piped_back ? elapsed(ev - 1, ev) : 0.0f);
  if (v.bounce) st.ms_copy = g_bounce_ms;  // the host threads' bounce copies
  return CWBL_OK;
}

}  // namespace

int set_last_error(int code, const char *msg) {
  g_err = msg;
  return code;
}

}  // namespace cwbl

using namespace cwbl;

extern "C" {

int cwbl_abi_version(void) { return CWBL_ABI_VERSION; }

const char *cwbl_last_error(void) { return g_err.c_str(); }

int cwbl_init(const cwbl_init_params *p) {
  if (!p) return fail(CWBL_ERR_ARG, "cwbl_init: null params");
  if (S.inited) release_all();
  if (p->nmember < 2) return fail(CWBL_ERR_ARG, "nmember must be >= 2 (got %d)", p->nmember);
  const int kp = supported_kp(p->nmember);
  if (kp < 0)
    return fail(CWBL_ERR_UNSUPPORTED, "nmember %d > %d not supported by this build",
                p->nmember, CWBL_MAX_MEMBERS);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(CWBL_ERR_NO_DEVICE, "no HIP device available (the core has no CPU path)");
  int dev = p->device;
  if (dev < 0) HIPCHK(hipGetDevice(&dev));
  if (dev >= ndev) return fail(CWBL_ERR_NO_DEVICE, "device %d >= device count %d", dev, ndev);
  HIPCHK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(CWBL_ERR_NO_DEVICE, "device %d is %s; this library is built for gfx950", dev,
                prop.gcnArchName);
  if (p->weight_function != 0 && p->weight_function != 1)
    return fail(CWBL_ERR_ARG, "weight_function must be 0 or 1");
  S.k = p->nmember;
  S.kp = kp;
  S.device = dev;
  S.wf = p->weight_function;
  S.norain = p->norain_value;
  S.q1_mode = p->q1_mode;
  S.ws_bytes = p->workspace_bytes ? p->workspace_bytes : (size_t(2) << 30);
  if (p->workspace_bytes) {
    S.handoff_budget = p->workspace_bytes;
  } else {  // 13 GB (98 304 points at k = 128), at most 40% of what is free now
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    S.handoff_budget = std::min<size_t>((size_t)13 << 30, fr / 10 * 4);
  }
  HIPCHK(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&S.sstream, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&S.h2d, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&S.d2h, hipStreamNonBlocking));
  {
    std::vector<double2> tab((size_t)4 * kQuadLevels * kQuadStride);  // 15, 23, 31, 63 nodes
    const int rounds[4] = {2, 3, 4, 8};
    for (int r = 0; r < 4; ++r)
      for (int l = 1; l <= kQuadLevels; ++l)
        quad_table(l, &tab[((size_t)r * kQuadLevels + (l - 1)) * kQuadStride],
                   8 * rounds[r] - 1);
    HIPCHK(S.quad.ensure(tab.size() * sizeof(double2)));
    HIPCHK(hipMemcpy(S.quad.p, tab.data(), tab.size() * sizeof(double2), hipMemcpyHostToDevice));
  }
  // path options (cwbl_set_option): every one back to its default
  S.jacobi = false;
  S.tq4 = 1;
  S.tq4_sub = 0;
  S.big_split = true;
  // (C4 per variable, r3: 32 k points 2.42 s, 16 k 2.47, 64 k 2.41, 96 k 2.39, 128 k 2.39)
  S.big_sub = 98304;
  S.binned = true;
  S.pageable_register = true;
  S.bin_div = 0;  // 0: by density (bin_div_for)
  S.lead_div = 0;
  S.serial_search = false;
#ifdef CWBL_DEBUG_KNOBS
  if (const char *e = std::getenv("CWBL_DEBUG_SERIAL")) S.serial_search = std::atoi(e) != 0;
#endif
  S.kp_natural = kp;
  select_kp();
  S.max_batch = 160000;
  S.max_batch_set = false;
  S.info_window = 1LL << 25;
  S.inited = true;
  return CWBL_OK;
}

int cwbl_set_option(int option, long long value) {
  if (!S.inited) return fail(CWBL_ERR_STATE, "cwbl_set_option before cwbl_init");
  auto range = [&](long long lo, long long hi) { return value >= lo && value <= hi; };
  switch (option) {
    case CWBL_OPT_SOLVER:
      if (!range(0, 1)) break;
      if (value == 1 && S.kp_natural > kMaxWaveKP)
        return fail(CWBL_ERR_UNSUPPORTED, "the Jacobi solver supports k <= %d", kMaxWaveKP);
      S.jacobi = value == 1;
      select_kp();
      return CWBL_OK;
    case CWBL_OPT_SPLIT40:
      if (!range(0, 1)) break;
      S.tq4 = (int)value;
      select_kp();
      return CWBL_OK;
    case CWBL_OPT_SPLIT40_BATCH:
      if (!range(0, 1 << 19)) break;
      S.tq4_sub = value;
      return CWBL_OK;
    case CWBL_OPT_SEARCH:
      if (!range(0, 1)) break;
      S.binned = value == 0;
      return CWBL_OK;
    case CWBL_OPT_BIG_PATH:
      if (!range(0, 1)) break;
      S.big_split = value == 1;
      return CWBL_OK;
    case CWBL_OPT_BIG_BATCH:
      if (!range(64, 1LL << 24)) break;
      S.big_sub = value;
      return CWBL_OK;
    case CWBL_OPT_PAGEABLE:
      if (!range(0, 1)) break;
      S.pageable_register = value == 0;
      return CWBL_OK;
    case CWBL_OPT_BIN_DIV:
      if (!range(0, 8)) break;
      S.bin_div = (int)value;
      return CWBL_OK;
    case CWBL_OPT_LEAD_DIV:
      if (!range(0, 1 << 20)) break;
      S.lead_div = (int)value;
      return CWBL_OK;
    case CWBL_OPT_MAX_BATCH:
      if (value != 0 && !range(256, 1LL << 31)) break;
      S.max_batch = value ? value : 160000;
      S.max_batch_set = value != 0;  // an explicit cap is used as given
      return CWBL_OK;
    case CWBL_OPT_INFO_WINDOW:
      if (value != 0 && !range(256, 1LL << 30)) break;
      S.info_window = value ? value : (1LL << 25);
      return CWBL_OK;
    default:
      return fail(CWBL_ERR_ARG, "cwbl_set_option: unknown option %d", option);
  }
  return fail(CWBL_ERR_ARG, "cwbl_set_option: value %lld out of range for option %d", value,
              option);
}

int cwbl_set_stream(void *stream) {
  if (int rc = require_device()) return rc;
  S.caller_stream = static_cast<hipStream_t>(stream);
  return CWBL_OK;
}

int cwbl_set_kernel_timing(int enable) {
  if (int rc = require_device()) return rc;
  S.ktiming = enable != 0;
  for (KTime &t : S.ktime) t = KTime{};
  return CWBL_OK;
}

int cwbl_kernel_times(cwbl_kernel_time *out, int cap, int *n) {
  if (int rc = require_device()) return rc;
  if (!n || cap < 0 || (cap > 0 && !out)) return fail(CWBL_ERR_ARG, "cwbl_kernel_times: bad arguments");
  int m = 0;
  for (int id = 0; id < KT_COUNT; ++id) {
    const KTime &t = S.ktime[id];
    if (t.launches == 0) continue;
    if (m < cap) {
      cwbl_kernel_time &o = out[m];
      std::memset(&o, 0, sizeof o);
      std::snprintf(o.name, sizeof o.name, "%s", kernel_name(id).c_str());
      o.launches = t.launches;
      o.points = t.points;
      o.ms = t.ms;
    }
    ++m;
  }
  *n = m;
  return CWBL_OK;
}

int cwbl_finalize(void) {
  if (S.inited) {
    (void)hipStreamSynchronize(S.stream);
    release_all();
  }
  return CWBL_OK;
}

int cwbl_set_obs(const cwbl_obs_set *o) {
  if (int rc = require_device()) return rc;
  if (!o) return fail(CWBL_ERR_ARG, "null obs set");
  if (o->n_gts < 0 || o->n_radar < 0 || (o->n_gts && !o->gts) || (o->n_radar && !o->radar))
    return fail(CWBL_ERR_ARG, "bad obs set counts/pointers");
  release_obs();
  const int mem = o->memory;
  if (mem == CWBL_MEM_DEVICE) HIPCHK(order_after_caller());
  const size_t k = (size_t)S.k;
  bool seen_g[CWBL_NUM_GTS_TYPES + 1] = {}, seen_r[CWBL_NUM_RADAR_TYPES + 1] = {};
  for (int e = 0; e < o->n_gts; ++e) {
    const cwbl_gts_obs &g = o->gts[e];
    if (g.type_id < 1 || g.type_id > CWBL_NUM_GTS_TYPES || seen_g[g.type_id])
      return fail(CWBL_ERR_ARG, "gts entry %d: bad or duplicate type_id %d", e, g.type_id);
    if (g.nvar < 1 || g.nvar > CWBL_MAX_NVAR || g.nobs < 0)
      return fail(CWBL_ERR_ARG, "gts type %d: bad nvar/nobs", g.type_id);
    if (g.nobs > 0 && (!g.xyz || !g.obs || !g.error || !g.hdxb || !g.qc))
      return fail(CWBL_ERR_ARG, "gts type %d: null array", g.type_id);
    seen_g[g.type_id] = true;
    S.obs.emplace_back();
    ObsType &t = S.obs.back();
    t.family = 0; t.type_id = g.type_id; t.nvar = g.nvar; t.nobs = g.nobs;
    const size_t n = (size_t)g.nobs, nv = (size_t)g.nvar;
    t.xyz.resize(3 * n);
    if (n) {
      if (mem == CWBL_MEM_DEVICE)
        HIPCHK(hipMemcpyAsync(t.xyz.data(), g.xyz, 3 * n * 4, hipMemcpyDeviceToHost, S.stream));
      else
        std::memcpy(t.xyz.data(), g.xyz, 3 * n * 4);
    }
    HIPCHK(stage(t.obs, g.obs, n * nv * 4, mem));
    HIPCHK(stage(t.error, g.error, n * nv * 4, mem));
    HIPCHK(stage(t.hdxb, g.hdxb, n * nv * k * 4, mem));
    HIPCHK(stage(t.qc, g.qc, n * nv * k * 4, mem));
  }
  for (int e = 0; e < o->n_radar; ++e) {
    const cwbl_radar_obs &r = o->radar[e];
    if (r.type_id < 1 || r.type_id > CWBL_NUM_RADAR_TYPES || seen_r[r.type_id])
      return fail(CWBL_ERR_ARG, "radar entry %d: bad or duplicate type_id %d", e, r.type_id);
    if (r.nobs < 0) return fail(CWBL_ERR_ARG, "radar type %d: bad nobs", r.type_id);
    if (r.nobs > 0 && (!r.xyz || !r.obs || !r.hdxb))
      return fail(CWBL_ERR_ARG, "radar type %d: null array", r.type_id);
    seen_r[r.type_id] = true;
    S.obs.emplace_back();
    ObsType &t = S.obs.back();
    t.family = 1; t.type_id = r.type_id; t.nvar = 1; t.nobs = r.nobs;
    const size_t n = (size_t)r.nobs;
    t.xyz.resize(3 * n);
    if (n) {
      if (mem == CWBL_MEM_DEVICE)
        HIPCHK(hipMemcpyAsync(t.xyz.data(), r.xyz, 3 * n * 4, hipMemcpyDeviceToHost, S.stream));
      else
        std::memcpy(t.xyz.data(), r.xyz, 3 * n * 4);
    }
    HIPCHK(stage(t.obs, r.obs, n * 4, mem));
    HIPCHK(stage(t.hdxb, r.hdxb, n * k * 4, mem));
  }
  HIPCHK(hipStreamSynchronize(S.stream));
  S.have_obs = true;
  return CWBL_OK;
}

int cwbl_analyze_var(const cwbl_var_params *vp, const cwbl_slab *sl, cwbl_stats *stats) {
  if (int rc = require_device()) return rc;
  if (!S.have_obs) return fail(CWBL_ERR_STATE, "cwbl_set_obs has not been called");
  if (!vp || !sl) return fail(CWBL_ERR_ARG, "null argument");
  if (sl->nx < 0 || sl->ny < 0 || sl->nz < 0 || sl->ix_lim < 0 || sl->iy_lim < 0 ||
      sl->ix_lim > sl->nx || sl->iy_lim > sl->ny || sl->ix_lim > sl->alt_nx ||
      sl->iy_lim > sl->alt_ny)
    return fail(CWBL_ERR_ARG, "slab bounds: nx=%d ny=%d ix_lim=%d iy_lim=%d alt=%dx%d",
                sl->nx, sl->ny, sl->ix_lim, sl->iy_lim, sl->alt_nx, sl->alt_ny);
  if (!(vp->multi_infl > 0.0f)) return fail(CWBL_ERR_ARG, "multi_infl must be > 0");
  if (sl->memory == CWBL_MEM_DEVICE) HIPCHK(order_after_caller());
  const auto t_start = std::chrono::steady_clock::now();
  S.kpend.clear();  // (an earlier call that failed midway leaves nothing to collect)
  S.kev_used = 0;
  g_bounce_ms = 0.0;
  cwbl_stats st;
  std::memset(&st, 0, sizeof st);
  const long long npts = (long long)sl->ix_lim * sl->iy_lim * sl->nz;
  if (npts >= (1LL << 32))  // the kernels enumerate a slab's points in 32 bits
    return fail(CWBL_ERR_ARG, "slab of %lld points: at most 2^32 - 1 per call", npts);
  st.points = npts;
  auto finish = [&]() {
    st.ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (stats) *stats = st;
    return CWBL_OK;
  };

  VarCall v;
  v.vp = vp;
  v.sl = sl;
  v.npts = npts;
  struct Unregister {  // a page-locked-in-place var, on every return path, once no queued
    VarCall &v;        // copy can still touch it
    ~Unregister() {
      if (!v.registered) return;
      (void)hipStreamSynchronize(S.h2d);
      (void)hipStreamSynchronize(S.d2h);
      (void)hipStreamSynchronize(S.stream);
      (void)hipGetLastError();
      (void)hipHostUnregister(v.sl->var);
    }
  } unreg{v};

  hipEvent_t e0, e1, e2, e_ready;
  HIPCHK(event(0, &e0));
  HIPCHK(hipEventRecord(e0, S.stream));
  if (int rc = plan_trees(v)) return rc;
  st.ntrees = v.nt;
  if (v.nt == 0 || npts == 0) {  // `if(all(.not. succeed)) cycle` (:66)
    HIPCHK(hipStreamSynchronize(S.stream));
    return finish();
  }
  for (const TreeDesc &d : v.descs) st.q1_undefined += d.q1_undef ? npts : 0;
  HIPCHK(event(1, &e1));
  HIPCHK(hipEventRecord(e1, S.stream));
  HIPCHK(event(2, &e2));
  if (int rc = stage_slab(v)) return rc;
  HIPCHK(hipEventRecord(e2, S.stream));
  plan_batches(v);
  if (int rc = stage_bounce(v)) return rc;
  if (int rc = alloc_call_buffers(v)) return rc;
  HIPCHK(event(3, &e_ready));  // inputs staged and the counters cleared
  HIPCHK(hipEventRecord(e_ready, S.stream));
  HIPCHK(hipStreamWaitEvent(S.sstream, e_ready, 0));

  // The searches run on S.sstream into two list buffers, the solves on S.stream: batch b + 1's
  // search (latency-bound, integer / fp32) overlaps batch b's solve (FP64-bound).  Search b
  // waits for the inputs and for the solve of b - 2 (same buffer); solve b waits for search b.
  const long long nbat = (long long)v.plan.size();
  for (long long bi = 0; bi < nbat; ++bi) {
    const long long g0 = v.plan[bi].first;
    const int nb = v.plan[bi].second;
    if (g0 + nb - v.win0 > v.info_cap) {  // close the info window; S.stream orders the reuse
      HIPCHK(launch_reduce_info(S.stream, S.info.as<int2>(), (int)(g0 - v.win0),
                                S.stats.as<DevStats>()));
      v.win0 = g0;
    }
    int2 *const infob = S.info.as<int2>() + (g0 - v.win0);  // this batch's info
    int *ncnt = (bi & 1) ? S.nbr_cnt2.as<int>() : S.nbr_cnt.as<int>();
    int *nidx = (bi & 1) ? S.nbr_idx2.as<int>() : S.nbr_idx.as<int>();
    const int ev = v.ev;
    hipEvent_t a, b, b2, dn;
    HIPCHK(event(ev, &a));
    HIPCHK(event(ev + 1, &b));
    HIPCHK(event(ev + 2, &b2));
    HIPCHK(event(ev + 3, &dn));
    if (int rc = search_batch(v, bi, ncnt, nidx, a, b)) return rc;
    HIPCHK(hipStreamWaitEvent(S.stream, b, 0));
    if (v.piped)
      if (int rc = upload_batch_var(v, bi)) return rc;
    HIPCHK(hipEventRecord(b2, S.stream));
    if (int rc = solve_batch_path(v, g0, nb, ncnt, nidx, infob, b2, dn)) return rc;
    HIPCHK(hipEventRecord(dn, S.stream));  // this batch's lists are free again
    if (v.piped_back)
      if (int rc = return_batch_var(v, bi, dn)) return rc;
    if (v.bounce && v.piped) {  // host side while the GPU works: next batch in, bi - 2 out
      if (bi + 1 < nbat)
        if (int rc = bounce_fill(v, bi + 1)) return rc;
      if (v.piped_back && bi >= State::kSlots - 1)
        if (int rc = bounce_drain(v, bi - (State::kSlots - 1))) return rc;
    }
    v.search_ev.push_back({ev, ev + 1});
    v.solve_ev.push_back({ev + 2, ev + 3});
    v.done_ev.push_back(ev + 3);
    v.ev += 4;
  }
  if (int rc = finish_call(v, st)) return rc;
  return finish();
}

int cwbl_solve_batch(int npts, const long long *col_off, const float *yo, const float *yb,
                     const float *xb, float inflat, int use_rtpp, float rtpp_alpha,
                     int use_rtps, float rtps_alpha, float *xa, double *evals, int memory) {
  if (int rc = require_device()) return rc;
  if (npts < 0 || (npts > 0 && (!col_off || !xb || !xa)))
    return fail(CWBL_ERR_ARG, "cwbl_solve_batch: bad arguments");
  if (npts == 0) return CWBL_OK;
  const size_t k = (size_t)S.k;
  std::vector<long long> hoff;
  const long long *doff = col_off;
  long long ncol;
  if (memory == CWBL_MEM_DEVICE) {
    HIPCHK(order_after_caller());
    HIPCHK(hipMemcpyAsync(&ncol, col_off + npts, 8, hipMemcpyDeviceToHost, S.stream));
    HIPCHK(hipStreamSynchronize(S.stream));
  } else {
    ncol = col_off[npts];
    for (int i = 0; i < npts; ++i)
      if (col_off[i + 1] < col_off[i]) return fail(CWBL_ERR_ARG, "col_off not monotone");
  }
  if (ncol > 0 && (!yo || !yb)) return fail(CWBL_ERR_ARG, "cwbl_solve_batch: null yo/yb");
  const float *dyo = yo, *dyb = yb, *dxb = xb;
  float *dxa = xa;
  double *dev = evals;
  if (memory != CWBL_MEM_DEVICE) {
    HIPCHK(stage(S.bcol, col_off, (size_t)(npts + 1) * 8, memory));
    HIPCHK(stage(S.byo, yo, (size_t)ncol * 4, memory));
    HIPCHK(stage(S.byb, yb, (size_t)ncol * k * 4, memory));
    HIPCHK(stage(S.bxb, xb, (size_t)npts * k * 4, memory));
    HIPCHK(S.bxa.ensure((size_t)npts * k * 4));
    if (evals) HIPCHK(S.bev.ensure((size_t)npts * k * 8));
    doff = S.bcol.as<long long>(); dyo = S.byo.as<float>(); dyb = S.byb.as<float>();
    dxb = S.bxb.as<float>(); dxa = S.bxa.as<float>(); dev = evals ? S.bev.as<double>() : nullptr;
  }
  HIPCHK(S.info.ensure((size_t)npts * sizeof(int2)));
  SolveConsts c = solve_consts(inflat, use_rtpp, rtpp_alpha, use_rtps, rtps_alpha);
  // Eigenvalues (dsyevd's ascending eval, module_eigen.f90:48-56): from the tridiagonal T the
  // tq kernels form, by bisection (launch_tridiag_eigvals), at every k; CWBL_OPT_SOLVER = 1
  // (k <= 64) takes them from the Jacobi eigensolver instead.
  const bool jacobi = S.jacobi && S.kp <= kMaxWaveKP;
  double *tri = nullptr;
  if (dev && !jacobi) {
    HIPCHK(S.btri.ensure((size_t)npts * 2 * S.kp * sizeof(double)));
    tri = S.btri.as<double>();
  }
  if (S.kp > kMaxWaveKP)
    HIPCHK(launch_solve_tq_big(S.stream, S.kp, true, nullptr, c, SlabDev{}, 0, npts, nullptr,
                               nullptr, doff, dyo, dyb, dxb, dxa, S.info.as<int2>(), tri));
  else if (jacobi)
    HIPCHK(launch_solve_assembled(S.stream, S.kp, c, npts, doff, dyo, dyb, dxb, dxa, dev,
                                  S.info.as<int2>()));
  else
    HIPCHK(launch_solve_tq(S.stream, S.kp, true, nullptr, c, SlabDev{}, 0, npts, nullptr,
                           nullptr, doff, dyo, dyb, dxb, dxa, S.info.as<int2>(), tri));
  if (tri) HIPCHK(launch_tridiag_eigvals(S.stream, S.kp, S.k, npts, tri, dev));
  if (memory != CWBL_MEM_DEVICE) {
    HIPCHK(hipMemcpyAsync(xa, dxa, (size_t)npts * k * 4, hipMemcpyDeviceToHost, S.stream));
    if (evals)
      HIPCHK(hipMemcpyAsync(evals, dev, (size_t)npts * k * 8, hipMemcpyDeviceToHost, S.stream));
  }
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_pack_columns(const float *global, int nx, int ny, int nz, int px, int py,
                      float *send) {
  if (int rc = require_device()) return rc;
  if (nx < 0 || ny < 0 || nz < 0 || px < 1 || py < 1 || px > kMaxRankDim || py > kMaxRankDim ||
      (((long long)nx * ny * nz) > 0 && (!global || !send)))
    return fail(CWBL_ERR_ARG, "cwbl_pack_columns: bad arguments");
  Decomp d;
  make_decomp(d, nx, ny, nz, px, py);
  HIPCHK(order_after_caller());
  HIPCHK(launch_pack_columns(S.stream, global, d, send));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_unpack_columns(const float *recv, int nx, int ny, int nz, int px, int py,
                        float *global) {
  if (int rc = require_device()) return rc;
  if (nx < 0 || ny < 0 || nz < 0 || px < 1 || py < 1 || px > kMaxRankDim || py > kMaxRankDim ||
      (((long long)nx * ny * nz) > 0 && (!global || !recv)))
    return fail(CWBL_ERR_ARG, "cwbl_unpack_columns: bad arguments");
  Decomp d;
  make_decomp(d, nx, ny, nz, px, py);
  HIPCHK(order_after_caller());
  HIPCHK(launch_unpack_columns(S.stream, recv, d, global));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_pack_members(const float *global, long long gstride, int nm, int nx, int ny, int nz,
                      int px, int py, float *send, long long sstride) {
  if (int rc = require_device()) return rc;
  const long long n = (long long)nx * ny * nz;
  if (nx < 0 || ny < 0 || nz < 0 || px < 1 || py < 1 || px > kMaxRankDim || py > kMaxRankDim ||
      nm < 0 || nm > 65535 || (nm > 1 && (gstride < n || sstride < n)) ||
      (n > 0 && nm > 0 && (!global || !send)))
    return fail(CWBL_ERR_ARG, "cwbl_pack_members: bad arguments");
  Decomp d;
  make_decomp(d, nx, ny, nz, px, py);
  HIPCHK(order_after_caller());
  HIPCHK(launch_transpose_columns(S.stream, false, global, gstride, nm, d, send, sstride));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_unpack_members(const float *recv, long long rstride, int nm, int nx, int ny, int nz,
                        int px, int py, float *global, long long gstride) {
  if (int rc = require_device()) return rc;
  const long long n = (long long)nx * ny * nz;
  if (nx < 0 || ny < 0 || nz < 0 || px < 1 || py < 1 || px > kMaxRankDim || py > kMaxRankDim ||
      nm < 0 || nm > 65535 || (nm > 1 && (gstride < n || rstride < n)) ||
      (n > 0 && nm > 0 && (!global || !recv)))
    return fail(CWBL_ERR_ARG, "cwbl_unpack_members: bad arguments");
  Decomp d;
  make_decomp(d, nx, ny, nz, px, py);
  HIPCHK(order_after_caller());
  HIPCHK(launch_transpose_columns(S.stream, true, recv, rstride, nm, d, global, gstride));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_vcoord_mean(const float *ph, long long n2d, int nz_ph, int k, int stagger, float g,
                     float *alt) {
  if (int rc = require_device()) return rc;
  if (n2d < 0 || k < 1 || (stagger != 0 && stagger != 1) || nz_ph < (stagger == 0 ? 2 : 1) ||
      (n2d > 0 && (!ph || !alt)))
    return fail(CWBL_ERR_ARG, "cwbl_vcoord_mean: bad arguments");
  // alpha = 1.0/(g*nmember) in default real (module_mpi_util.f90:496)
  const float gk = g * (float)k;
  const float alpha = 1.0f / gk;
  HIPCHK(order_after_caller());
  HIPCHK(launch_vcoord_mean(S.stream, ph, n2d, nz_ph, k, stagger, alpha, alt));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_member_sum(const float *fields, long long n, int nm, float *out) {
  if (int rc = require_device()) return rc;
  if (n < 0 || nm < 1 || (n > 0 && (!fields || !out)))
    return fail(CWBL_ERR_ARG, "cwbl_member_sum: bad arguments");
  HIPCHK(order_after_caller());
  HIPCHK(launch_member_sum(S.stream, fields, n, nm, out));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_scale(float *x, long long n, float alpha) {
  if (int rc = require_device()) return rc;
  if (n < 0 || (n > 0 && !x)) return fail(CWBL_ERR_ARG, "cwbl_scale: bad arguments");
  HIPCHK(order_after_caller());
  HIPCHK(launch_scale(S.stream, x, n, alpha));
  HIPCHK(hipStreamSynchronize(S.stream));
  return CWBL_OK;
}

int cwbl_search(int nobs, const float *obs_xyz, float hclr, float vclr, int max_lz_pts,
                int nq, const float *q_xyz, int *nfound, int *idx, float *r2, int memory) {
  if (int rc = require_device()) return rc;
  if (nobs < 0 || nq < 0 || max_lz_pts < 1 || !(hclr > 0.0f))
    return fail(CWBL_ERR_ARG, "cwbl_search: bad arguments");
  if (memory == CWBL_MEM_DEVICE)
    return fail(CWBL_ERR_UNSUPPORTED, "cwbl_search takes host arrays");
  const float hinv = 1.0f / (hclr * 1e3f);
  const float vinv = vclr > 0.0f ? 1.0f / (vclr * 1e3f) : -1.0f;
  const bool dim3 = vinv > 0.0f;
  std::vector<float> nx(3 * (size_t)nobs);
  for (int j = 0; j < nobs; ++j) {
    nx[3 * j] = obs_xyz[3 * j] * hinv;
    nx[3 * j + 1] = obs_xyz[3 * j + 1] * hinv;
    nx[3 * j + 2] = dim3 ? obs_xyz[3 * j + 2] * vinv : -1.0f;
  }
  TreeBufs tb;
  build_kdtree(nx.data(), nobs, dim3 ? 3 : 2, tb.host);
  tb.depth = tree_depth(tb.host);
  if (tb.depth >= kSearchStackDepth)
    return fail(CWBL_ERR_UNSUPPORTED, "k-d tree too deep");
  const HostTree &h = tb.host;
  HIPCHK(tb.nodes.ensure(std::max<size_t>(h.nodes.size(), 1) * sizeof(TreeNode)));
  HIPCHK(tb.rdata.ensure(h.rdata.size() * sizeof(float)));
  HIPCHK(tb.ind.ensure(h.ind.size() * sizeof(int) + 4));
  if (!h.nodes.empty())
    HIPCHK(hipMemcpyAsync(tb.nodes.p, h.nodes.data(), h.nodes.size() * sizeof(TreeNode),
                          hipMemcpyHostToDevice, S.stream));
  HIPCHK(hipMemcpyAsync(tb.rdata.p, h.rdata.data(), h.rdata.size() * sizeof(float),
                        hipMemcpyHostToDevice, S.stream));
  if (nobs)
    HIPCHK(hipMemcpyAsync(tb.ind.p, h.ind.data(), h.ind.size() * sizeof(int),
                          hipMemcpyHostToDevice, S.stream));
  TreeDesc d{};
  d.nodes = tb.nodes.as<TreeNode>();
  d.rdata = tb.rdata.as<float4>();
  d.ind = tb.ind.as<int>();
  d.hclr_inv = hinv;
  d.vclr_inv = vinv;
  d.tree_dim = dim3 ? 3 : 2;
  d.query3d = dim3 ? 1 : 0;
  d.nvar = 1;
  d.max_lz = nobs > 0 ? max_lz_pts : 0;
  d.list_off = 0;
  DevBuf dd;
  HIPCHK(dd.ensure(sizeof d));
  HIPCHK(hipMemcpyAsync(dd.p, &d, sizeof d, hipMemcpyHostToDevice, S.stream));
  HIPCHK(stage(S.qxyz, q_xyz, (size_t)nq * 12, CWBL_MEM_HOST));
  HIPCHK(S.qnf.ensure((size_t)nq * 4));
  HIPCHK(S.qidx.ensure((size_t)nq * max_lz_pts * 4));
  HIPCHK(S.qr2.ensure((size_t)nq * max_lz_pts * 4));
  HIPCHK(launch_search_single(S.stream, dd.as<TreeDesc>(), tb.depth, search_r2(), nq,
                              S.qxyz.as<float>(),
                              max_lz_pts, S.qnf.as<int>(), S.qidx.as<int>(), S.qr2.as<float>()));
  HIPCHK(hipMemcpyAsync(nfound, S.qnf.p, (size_t)nq * 4, hipMemcpyDeviceToHost, S.stream));
  HIPCHK(hipMemcpyAsync(idx, S.qidx.p, (size_t)nq * max_lz_pts * 4, hipMemcpyDeviceToHost,
                        S.stream));
  HIPCHK(hipMemcpyAsync(r2, S.qr2.p, (size_t)nq * max_lz_pts * 4, hipMemcpyDeviceToHost,
                        S.stream));
  HIPCHK(hipStreamSynchronize(S.stream));
  dd.release();
  tb.nodes.release(); tb.rdata.release(); tb.ind.release();
  return CWBL_OK;
}

}  // extern "C"
