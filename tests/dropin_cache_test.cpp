// Unit test of hb_mcmc_amd/csrc/hb_dropin.hpp (the drop-in's exact context
// cache, logL memo and call combiner), built with plain g++ by
// tests/test_dropin_cache.py -- no HIP, no GPU.  The "context" is a fake that
// counts its creations and evaluates a cheap deterministic function of the
// parameters; prints "ok" and exits 0 when every check passes.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../hb_mcmc_amd/csrc/hb_dropin.hpp"

using namespace hbdrop;

struct Fake {
  std::vector<double> f;  // its light curve's fluxes: the "model" reads them
  std::atomic<int> evals{0};
};

static int g_created = 0, g_destroyed = 0;
static std::atomic<int> g_batches{0};

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

static double model(const Fake* c, const double* p) {
  double v = 0;
  for (int k = 0; k < kNPars; ++k) v += p[k] * (k + 1);
  return v + c->f[0];
}

static int g_eval_us = 0;  // a GPU round trip's duration (section 4)

static std::atomic<int> g_conc{0}, g_conc_max{0};

static int eval(Fake* c, int lane, const double* rows, int w, double* out, Times* tm) {
  const int k = ++g_conc;
  for (int m = g_conc_max; k > m && !g_conc_max.compare_exchange_weak(m, k);) {
  }
  if (lane < 0 || lane >= kMaxLanes) abort();
  if (g_eval_us) std::this_thread::sleep_for(std::chrono::microseconds(g_eval_us));
  for (int i = 0; i < w; ++i) out[i] = model(c, rows + (size_t)i * kNPars);
  c->evals += w;
  ++g_batches;
  --g_conc;
  tm->upload = tm->launch = tm->download = 0;
  return 0;
}

static uint64_t same_key(const double*, const double*, const double*, long, const double*, const double*) {
  return 7;
}

int main() {
  Cache<Fake> cache(
      [](const double*, const double* f, const double*, long n, const double*, const double*) {
        ++g_created;
        Fake* c = new Fake;
        c->f.assign(f, f + n);
        return c;
      },
      [](Fake* c) {
        ++g_destroyed;
        delete c;
      },
      3);
  const long n = 64;
  std::vector<double> t(n), f1(n), f2(n), s(n, 1e-3);
  for (long i = 0; i < n; ++i) t[i] = 0.01 * i, f1[i] = 1.0 + 1e-3 * i, f2[i] = f1[i];
  f2[17] = nextafter(f2[17], 2.0);  // one ulp apart: a different light curve
  const double mag[5] = {1000, 1, 1, 1, 1}, err[4] = {1e15, 1e15, 1e15, 1e15};

  // 1. the same arrays (same pointers, then copies at other addresses) -> one context
  auto a = cache.get(t.data(), f1.data(), s.data(), n, mag, err);
  auto a2 = cache.get(t.data(), f1.data(), s.data(), n, mag, err);
  std::vector<double> tc(t), fc(f1), sc(s);
  auto a3 = cache.get(tc.data(), fc.data(), sc.data(), n, mag, err);
  CHECK(a.get() == a2.get() && a.get() == a3.get() && g_created == 1);

  // 2. every light curve forced onto one hash key: f1 and f2 still get two
  //    contexts, and each lookup finds its own
  cache.set_hash(same_key);
  auto b = cache.get(t.data(), f2.data(), s.data(), n, mag, err);
  CHECK(b.get() != a.get() && g_created == 2);
  CHECK(cache.get(tc.data(), fc.data(), sc.data(), n, mag, err).get() == a.get());
  std::vector<double> f2c(f2);
  CHECK(cache.get(t.data(), f2c.data(), s.data(), n, mag, err).get() == b.get());
  // same pointers, contents changed in place: not the old context
  const double keep = f1[3];
  f1[3] = -5.0;
  auto c = cache.get(t.data(), f1.data(), s.data(), n, mag, err);
  CHECK(c.get() != a.get() && c.get() != b.get() && g_created == 3);
  f1[3] = keep;
  c.reset();  // idle now: the entry capacity 3 evicts next
  // magnitude data are part of the key
  const double mag2[5] = {1000, 1, 1, 1, 1.5};
  auto d = cache.get(t.data(), f1.data(), s.data(), n, mag2, err);
  CHECK(d.get() != a.get() && g_created == 4);
  cache.set_hash(nullptr);
  CHECK(cache.size() == 3 && g_destroyed == 1);

  // 3. memo: a repeated parameter vector is answered from the table; one
  //    flipped bit is a fresh evaluation
  Eval<Fake> ev = eval;
  double p[kNPars];
  for (int k = 0; k < kNPars; ++k) p[k] = 0.1 * (k + 1);
  double v1 = 0, v2 = 0, v3 = 0;
  CHECK(a->call(p, &v1, ev) == 0 && a->ctx->evals == 1);
  CHECK(a->call(p, &v2, ev) == 0 && a->ctx->evals == 1 && v2 == v1 && a->st.memo_hits == 1);
  double q[kNPars];
  memcpy(q, p, sizeof q);
  uint64_t bits;
  memcpy(&bits, &q[4], 8);
  bits ^= 1;  // lowest mantissa bit of the inclination
  memcpy(&q[4], &bits, 8);
  CHECK(a->call(q, &v3, ev) == 0 && a->ctx->evals == 2 && v3 == model(a->ctx, q));
  // the other light curve's memo is its own
  double vb = 0;
  CHECK(b->call(p, &vb, ev) == 0 && b->ctx->evals == 1 && vb == model(b->ctx, p));
  // LRU: kMemoCap fresh vectors push p out unless p is re-asked for
  for (int r = 0; r < kMemoCap + 10; ++r) {
    double z[kNPars];
    memcpy(z, p, sizeof z);
    z[0] = 1000.0 + r;
    double vz;
    CHECK(a->call(z, &vz, ev) == 0 && vz == model(a->ctx, z));
    if (r % 50 == 0) CHECK(a->call(q, &vz, ev) == 0 && vz == v3);  // q stays fresh
  }
  const int before = a->ctx->evals;
  CHECK(a->call(q, &v3, ev) == 0 && a->ctx->evals == before);      // still memoised
  CHECK(a->call(p, &v1, ev) == 0 && a->ctx->evals == before + 1);  // evicted, evaluated again

  // 4. combiner: 25 threads x 2 calls per "iteration" (x then y), like
  //    mcmc_wrapper2.c:488-489; every result exact, the x calls memo hits
  //    after the first iteration, and batches combine several callers --
  //    with the waiters sleeping at once, and with the spin / batch-window
  //    policy libhbmi can switch on, and with leaders chaining batches
  g_eval_us = 20;
  for (int pol = 0; pol < 7; ++pol) {
    std::vector<double> fp(f2);
    fp[0] += 1e-6 * (pol + 1);  // a fresh context per policy
    auto e = cache.get(t.data(), fp.data(), s.data(), n, mag, err);
    e->spin_s = pol >= 1 ? 200e-6 : 0.0;
    e->window_s = pol == 2 ? 30e-6 : 0.0;
    e->lanes = pol >= 3 ? 4 : 1;  // policy 3: four lanes with spinning, 4: four lanes, sleeping waiters
    if (pol == 4) e->spin_s = 0.0;
    if (pol >= 5) e->spin_s = 0.0, e->lanes = pol == 5 ? 1 : 2, e->chain = 4;  // leaders chain batches
    g_conc_max = 0;
    const int nth = 25, iters = 40;
    const int ev0 = e->ctx->evals;
    g_batches = 0;
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int j = 0; j < nth; ++j)
      th.emplace_back([&, j] {
        double x[kNPars];
        for (int k = 0; k < kNPars; ++k) x[k] = 0.01 * (j + 1) * (k + 1);
        for (int it = 0; it < iters; ++it) {
          double y[kNPars];
          memcpy(y, x, sizeof y);
          y[0] += 1e-3 * (it + 1);
          double lx, ly;
          if (e->call(x, &lx, ev) != 0 || lx != model(e->ctx, x)) ++bad;
          if (e->call(y, &ly, ev) != 0 || ly != model(e->ctx, y)) ++bad;
          if (it % 2 == 0) memcpy(x, y, sizeof x);  // "accepted"
        }
      });
    for (auto& x : th) x.join();
    CHECK(bad == 0);
    const int evals = e->ctx->evals - ev0;
    // first x of each thread + one y per iteration (y values are new states);
    // a thread descheduled while the others add kMemoCap states may find its
    // accepted y evicted and ask again (still the exact value)
    if (evals < nth + nth * iters || evals > nth + nth * iters + nth * iters / 10)
      fprintf(stderr, "policy %d: %d evaluations\n", pol, evals);
    CHECK(evals >= nth + nth * iters && evals <= nth + nth * iters + nth * iters / 10);
    CHECK(g_batches < evals);
    CHECK(e->st.calls == (uint64_t)(2 * nth * iters) && e->st.walkers == (uint64_t)evals);
    CHECK(g_conc_max <= e->lanes && (e->lanes == 1 || g_conc_max > 1));
    printf("policy %d: %d evaluations in %d batches, up to %d at once\n", pol, evals, (int)g_batches,
           (int)g_conc_max);
    CHECK(e->npending.load() == 0 && e->inflight.load() == 0 && e->lane_busy == 0 && e->pending.empty());
  }
  printf("ok\n");
  return 0;
}
