// hb_dropin.hpp -- host-side bookkeeping of the likelihood3.h drop-in
// (loglikelihood(), likelihood3.c:809-873), free of HIP so that it builds and
// is unit-tested with plain g++ (tests/test_dropin_cache.py).
//
// The reference sampler calls loglikelihood(t, f, sigma, N, params, mag,
// magerr) from 25 OpenMP threads, twice per chain per iteration
// (mcmc_wrapper2.c:383-489), always with the same light curve.  Three pieces
// turn that into few GPU round trips without changing any result:
//
//  * Cache: one resident context per light curve.  A light curve is the five
//    arrays bit for bit: a lookup first compares the stored copy with the
//    caller's arrays (memcmp; the caller passes the same pointers every call,
//    so the entry that last matched them is tried first), then falls back to a
//    64-bit hash over them -- and a hash hit is still compared in full, so two
//    light curves whose hashes collide get two contexts.
//  * Memo: per context, logL by the exact bytes of the 21 parameters.  The
//    first of a chain's two calls per iteration (:488, logLx[chain_id] of
//    x[chain_id]) re-evaluates a state the library has already evaluated --
//    the previous iteration's accepted y, or the unchanged x -- and gets the
//    same double back from the table: a walker's logL does not depend on the
//    batch it rides in (tests/test_gpu_parity.py batch-reversal and
//    fused-vs-two-launch tests).  LRU, kMemoCap entries (a chain that keeps
//    rejecting re-asks for its x every iteration, so it stays fresh).
//  * Combiner: concurrent misses on one context are evaluated as one batch.
//    A caller queues its parameters; if no batch is in flight it becomes the
//    leader, takes every queued request and runs them with one evaluation
//    (Eval); the others sleep until their result is written.  Requests that
//    arrive during a batch form the next one.
//
// Stats (calls, memo hits, batches, walkers, seconds spent combining, in the
// evaluation's upload / launch / download+sync, and waiters' wake-up latency)
// are kept per context; libhbmi writes them as JSON at exit when
// HBMI_DROPIN_STATS names a file (hbx_dropin_stats for the running totals).
#pragma once

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace hbdrop {

constexpr int kNPars = 21;  // likelihood3.h:26 (NPARS)
constexpr int kMemoCap = 256;
constexpr size_t kCacheMax = 8;  // resident light curves

inline uint64_t mix64(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  h *= 0xbf58476d1ce4e5b9ull;
  return h ^ (h >> 31);
}
// four independent lanes (the multiply chains overlap), folded at the end
inline uint64_t hash_doubles(uint64_t h, const double* a, long n) {
  uint64_t l[4] = {h, h ^ 0x1111, h ^ 0x2222, h ^ 0x3333};
  long i = 0;
  for (; i + 4 <= n; i += 4)
    for (int k = 0; k < 4; ++k) {
      uint64_t v;
      memcpy(&v, a + i + k, 8);
      l[k] = mix64(l[k], v);
    }
  for (; i < n; ++i) {
    uint64_t v;
    memcpy(&v, a + i, 8);
    l[0] = mix64(l[0], v);
  }
  return mix64(mix64(mix64(mix64(l[0], l[1]), l[2]), l[3]), (uint64_t)n);
}

using HashFn = uint64_t (*)(const double* t, const double* f, const double* s, long n, const double* mag,
                            const double* err);

inline uint64_t hash_light_curve(const double* t, const double* f, const double* s, long n, const double* mag,
                                 const double* err) {
  uint64_t k = hash_doubles(0x5eed, t, n);
  k = hash_doubles(k, f, n);
  k = hash_doubles(k, s, n);
  k = hash_doubles(k, mag, 5);
  return hash_doubles(k, err, 4);
}

// The arrays that define a resident context, kept bit for bit.
struct LightCurve {
  long n = 0;
  std::vector<double> t, f, s;
  double mag[5] = {0}, err[4] = {0};
  uint64_t hash = 0;

  void assign(const double* t_, const double* f_, const double* s_, long n_, const double* mag_,
              const double* err_, uint64_t h) {
    n = n_;
    t.assign(t_, t_ + n_);
    f.assign(f_, f_ + n_);
    s.assign(s_, s_ + n_);
    memcpy(mag, mag_, sizeof mag);
    memcpy(err, err_, sizeof err);
    hash = h;
  }
  bool equals(const double* t_, const double* f_, const double* s_, long n_, const double* mag_,
              const double* err_) const {
    const size_t b = sizeof(double) * (size_t)n_;
    return n == n_ && memcmp(mag, mag_, sizeof mag) == 0 && memcmp(err, err_, sizeof err) == 0 &&
           memcmp(t.data(), t_, b) == 0 && memcmp(f.data(), f_, b) == 0 && memcmp(s.data(), s_, b) == 0;
  }
};

// logL by the exact parameter bytes, least recently used entry replaced.
class Memo {
 public:
  explicit Memo(int cap = kMemoCap) : e_((size_t)cap) {}
  bool find(const double* p, double* v) {
    const uint64_t h = hash_doubles(0x9a9a, p, kNPars);
    for (Ent& e : e_)
      if (e.use && e.h == h && memcmp(e.p, p, sizeof e.p) == 0) {
        e.use = ++tick_;
        *v = e.v;
        return true;
      }
    return false;
  }
  void put(const double* p, double v) {
    const uint64_t h = hash_doubles(0x9a9a, p, kNPars);
    Ent* slot = &e_[0];
    for (Ent& e : e_) {
      if (e.use && e.h == h && memcmp(e.p, p, sizeof e.p) == 0) {  // already there (two callers, one state)
        slot = &e;
        break;
      }
      if (e.use < slot->use) slot = &e;  // unused (use 0) or least recently used
    }
    slot->h = h;
    memcpy(slot->p, p, sizeof slot->p);
    slot->v = v;
    slot->use = ++tick_;
  }
  void clear() {
    for (Ent& e : e_) e.use = 0;
  }

 private:
  struct Ent {
    uint64_t h = 0, use = 0;  // use 0: empty
    double p[kNPars];
    double v = 0;
  };
  std::vector<Ent> e_;
  uint64_t tick_ = 0;
};

struct Stats {
  uint64_t calls = 0, memo_hits = 0, batches = 0, walkers = 0, max_batch = 0;
  // seconds: the leader's staging of a batch's parameters; the evaluation's
  // upload, launch and download + wait (split by Eval, see Times); callers'
  // wake-up after their batch completed
  double s_combine = 0, s_upload = 0, s_launch = 0, s_download = 0, s_wake = 0;
  uint64_t waiters = 0;
};

// What an evaluation reports: seconds in its upload, launch and download +
// synchronisation (host clock).
struct Times {
  double upload = 0, launch = 0, download = 0;
};

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Evaluate w parameter rows (w x 21, row-major, in `params`) on evaluation
// lane `lane` into out[w]; returns 0 or an error code.  Lanes are independent
// (libhbmi: one context and stream each), so batches on different lanes may
// run at the same time.
template <class Ctx>
using Eval = std::function<int(Ctx*, int lane, const double* params, int w, double* out, Times* tm)>;
// A staging area of w x 21 doubles for lane `lane` that Eval reads in place
// (pinned memory), or nullptr for the entry's own vector.
template <class Ctx>
using Stage = std::function<double*(Ctx*, int lane, int w)>;

constexpr int kMaxLanes = 8;

template <class Ctx>
struct Entry {
  LightCurve lc;
  Ctx* ctx = nullptr;
  const double *pt = nullptr, *pf = nullptr, *ps = nullptr;  // the caller's pointers at the last match
  uint64_t last_use = 0;

  struct Req {
    const double* p = nullptr;
    double out = 0;
    int rc = 0;
    double t_done = 0;
    std::atomic<bool> done{false};
  };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req*> pending;
  std::atomic<int> npending{0};
  std::atomic<int> inflight{0};  // batches being evaluated (at most `lanes`)
  unsigned lane_busy = 0;        // bit k: lane k holds a batch (under mu)
  Memo memo;
  std::atomic<bool> use_memo{true};
  std::vector<double> params[kMaxLanes], out[kMaxLanes];  // per-lane staging (when Stage gives none)
  Stats st;
  std::atomic<uint64_t> wake_ns{0}, wake_n{0};  // callers answered in another caller's batch
  // Policy (set by the owner before use):
  //  * lanes: batches that may be in flight at once, each on its own lane;
  //    a caller that finds a free lane leads a batch right away instead of
  //    waiting for the running one to finish;
  //  * spin_s: a caller whose request rides in another caller's batch polls
  //    its done flag (lock released) this long before it sleeps on the
  //    condition variable;
  //  * window_s: a new leader waits up to this long for the queue to reach
  //    the largest batch of the last kWindowHist batches before it launches.
  //  * chain: a leader whose own request is answered leads up to this many
  //    further batches from the queue before it returns, so the next batch is
  //    launched at once instead of after a waiter wakes up.
  int lanes = 1;
  double spin_s = 0, window_s = 0;
  int chain = 0;
  static constexpr int kWindowHist = 16;
  int hist[kWindowHist] = {0};
  int nhist = 0;

  static void relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }

  // loglikelihood() of one parameter vector: memo, else combined evaluation.
  int call(const double* p, double* result, const Eval<Ctx>& eval, const Stage<Ctx>& stage = nullptr) {
    std::unique_lock<std::mutex> lk(mu);
    ++st.calls;
    if (use_memo && memo.find(p, result)) {
      ++st.memo_hits;
      return 0;
    }
    Req r;
    r.p = p;
    pending.push_back(&r);
    npending.store((int)pending.size(), std::memory_order_release);
    const int nl = lanes < 1 ? 1 : lanes > kMaxLanes ? kMaxLanes : lanes;
    bool spun = false;
    int led = 0;  // batches this caller led
    for (;;) {
      const bool can_lead = inflight.load(std::memory_order_relaxed) < nl && !pending.empty();
      if (r.done.load(std::memory_order_acquire) && !(can_lead && led > 0 && led <= chain)) {
        if (led == 0) {
          wake_ns.fetch_add((uint64_t)((now_s() - r.t_done) * 1e9), std::memory_order_relaxed);
          wake_n.fetch_add(1, std::memory_order_relaxed);
        }
        *result = r.out;
        return r.rc;
      }
      if (can_lead) {  // lead a batch on a free lane
        ++led;
        int lane = 0;
        while (lane_busy >> lane & 1u) ++lane;
        lane_busy |= 1u << lane;
        inflight.fetch_add(1, std::memory_order_relaxed);
        int target = 0;
        for (int i = 0; i < nhist; ++i) target = hist[i] > target ? hist[i] : target;
        if (window_s > 0 && (int)pending.size() < target) {
          lk.unlock();
          const double t_end = now_s() + window_s;
          for (int k = 1; npending.load(std::memory_order_acquire) < target; ++k) {
            if ((k & 15) == 0 && now_s() > t_end) break;
            relax();
          }
          lk.lock();
        }
        std::vector<Req*> batch;
        batch.swap(pending);
        npending.store(0, std::memory_order_release);
        lk.unlock();
        const double t0 = now_s();
        const int w = (int)batch.size();
        double* rows = stage ? stage(ctx, lane, w) : nullptr;
        if (!rows) {
          params[lane].resize((size_t)w * kNPars);
          rows = params[lane].data();
        }
        out[lane].resize((size_t)w);
        for (int i = 0; i < w; ++i) memcpy(rows + (size_t)i * kNPars, batch[(size_t)i]->p, kNPars * sizeof(double));
        const double t1 = now_s();
        Times tm;
        const int rc = eval(ctx, lane, rows, w, out[lane].data(), &tm);
        lk.lock();
        const double t2 = now_s();
        for (int i = 0; i < w; ++i) {
          Req* q = batch[(size_t)i];
          q->out = out[lane][(size_t)i];
          q->rc = rc;
          q->t_done = t2;
          if (rc == 0 && use_memo) memo.put(q->p, q->out);
          q->done.store(true, std::memory_order_release);  // q may return (and its Req vanish) from here on
        }
        hist[nhist < kWindowHist ? nhist++ : (int)(st.batches % kWindowHist)] = w;
        ++st.batches;
        st.walkers += (uint64_t)w;
        if ((uint64_t)w > st.max_batch) st.max_batch = (uint64_t)w;
        st.s_combine += t1 - t0;
        st.s_upload += tm.upload;
        st.s_launch += tm.launch;
        st.s_download += tm.download;
        lane_busy &= ~(1u << lane);
        inflight.fetch_sub(1, std::memory_order_relaxed);
        cv.notify_all();
        continue;  // own request done (it was in the first batch): returns above, or chains
      }
      if (spin_s > 0 && !spun) {  // poll first, sleep after
        spun = true;
        lk.unlock();
        const double t_end = now_s() + spin_s;
        for (int k = 1; !r.done.load(std::memory_order_acquire) && inflight.load(std::memory_order_relaxed) >= nl;
             ++k) {
          if ((k & 63) == 0) {
            if (now_s() > t_end) break;
            std::this_thread::yield();
          }
          relax();
        }
        lk.lock();
        continue;
      }
      cv.wait(lk);
    }
  }
};

// The resident contexts, shared by every caller thread.
template <class Ctx>
class Cache {
 public:
  using Create = std::function<Ctx*(const double* t, const double* f, const double* s, long n, const double* mag,
                                    const double* err)>;
  using Destroy = std::function<void(Ctx*)>;
  using Init = std::function<void(Entry<Ctx>&)>;  // policy of a new entry, before anyone sees it

  Cache(Create create, Destroy destroy, size_t max = kCacheMax, Init init = nullptr)
      : create_(std::move(create)), destroy_(std::move(destroy)), init_(std::move(init)), max_(max) {}

  // test hook: replace the light-curve hash (nullptr restores the default)
  void set_hash(HashFn h) { hash_ = h ? h : hash_light_curve; }

  std::shared_ptr<Entry<Ctx>> get(const double* t, const double* f, const double* s, long n, const double* mag,
                                  const double* err) {
    std::lock_guard<std::mutex> lk(mu_);
    // the caller's own arrays again (the sampler's case): compare in full
    for (auto& e : ents_)
      if (e->pt == t && e->pf == f && e->ps == s && e->lc.equals(t, f, s, n, mag, err)) return touch(e);
    const uint64_t key = hash_(t, f, s, n, mag, err);
    for (auto& e : ents_)
      if (e->lc.hash == key && e->lc.equals(t, f, s, n, mag, err)) {
        e->pt = t, e->pf = f, e->ps = s;
        return touch(e);
      }
    if (ents_.size() >= max_) {  // evict the least recently used idle entry
      size_t victim = ents_.size();
      for (size_t i = 0; i < ents_.size(); ++i)
        if (ents_[i].use_count() == 1 && (victim == ents_.size() || ents_[i]->last_use < ents_[victim]->last_use))
          victim = i;
      if (victim < ents_.size()) {
        destroy_(ents_[victim]->ctx);
        ents_.erase(ents_.begin() + (long)victim);
      }
    }
    auto e = std::make_shared<Entry<Ctx>>();
    e->ctx = create_(t, f, s, n, mag, err);
    if (!e->ctx) return nullptr;
    e->lc.assign(t, f, s, n, mag, err, key);
    e->pt = t, e->pf = f, e->ps = s;
    if (init_) init_(*e);
    ents_.push_back(e);
    ++created_;
    return touch(e);
  }

  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return ents_.size();
  }
  uint64_t created() {
    std::lock_guard<std::mutex> lk(mu_);
    return created_;
  }
  // a snapshot of every resident entry (for stats)
  std::vector<std::shared_ptr<Entry<Ctx>>> entries() {
    std::lock_guard<std::mutex> lk(mu_);
    return ents_;
  }

 private:
  std::shared_ptr<Entry<Ctx>> touch(std::shared_ptr<Entry<Ctx>>& e) {
    e->last_use = ++tick_;
    return e;
  }
  std::mutex mu_;
  std::vector<std::shared_ptr<Entry<Ctx>>> ents_;
  Create create_;
  Destroy destroy_;
  Init init_;
  size_t max_;
  HashFn hash_ = hash_light_curve;
  uint64_t tick_ = 0, created_ = 0;
};

}  // namespace hbdrop
