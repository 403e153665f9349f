"""The device-resident sampler (hb_mcmc_amd/csrc/hb_dsampler.hip): the same
PT-MCMC loop as the host sampler with proposals, walls, priors, Hastings,
history and tempering swaps on the GPU.

CPU: the level-parallel replay of the W sequential tempering attempts equals
the sequential ptmcmc loop (mcmc_wrapper2.c:768-817) on random inputs -- the
schedule logic of hb_dsampler_step restated in numpy.

GPU: (1) the device run reproduces the REFERENCE sampler's own trace
(`HB_MCMC 1200 127079833 0.5021 0`, tests/golden) like the host loop does:
states and bookkeeping exact, logL within 1e-10; (2) after K iterations the
device sampler's whole state (states, logL, chain ids, RNG streams, history,
counters) equals the host sampler's after the same K iterations with the same
GPU likelihood, bit for bit -- at W = 50 (trace config) and W = 4096 with the
large-W ladder, past NPAST so differential-evolution jumps are exercised.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def levels(b, W):
    """Dependency level of each attempt (hb_dsampler_step); -1 = void (b = W-1)."""
    last = np.zeros(W + 1, dtype=np.int64)
    lv = np.full(len(b), -1)
    for i, x in enumerate(b):
        if x + 1 >= W:
            continue
        lv[i] = max(last[x], last[x + 1]) + 1
        last[x] = last[x + 1] = lv[i]
    return lv


def swap_sequential(idx, L, temp, b, beta):
    idx = idx.copy()
    for x, be in zip(b, beta):
        a = x + 1
        if a >= len(idx):
            continue
        olda, oldb = idx[a], idx[x]
        hs = (temp[x] - temp[a]) / (temp[x] * temp[a])
        if np.exp((L[oldb] - L[olda]) * hs) >= be:
            idx[a], idx[x] = oldb, olda
    return idx


def swap_levels(idx, L, temp, b, beta):
    idx = idx.copy()
    lv = levels(b, len(idx))
    for level in range(1, lv.max() + 1):
        sel = np.nonzero(lv == level)[0]
        xs = b[sel]
        assert len(np.unique(np.concatenate([xs, xs + 1]))) == 2 * len(xs), "attempts of a level overlap"
        a = xs + 1
        olda, oldb = idx[a], idx[xs]
        hs = (temp[xs] - temp[a]) / (temp[xs] * temp[a])
        acc = np.exp((L[oldb] - L[olda]) * hs) >= beta[sel]
        idx[a[acc]], idx[xs[acc]] = oldb[acc], olda[acc]
    return idx


@pytest.mark.parametrize("W", [2, 3, 50, 1000, 4096])
def test_level_schedule_equals_sequential_swaps(W):
    rng = np.random.default_rng(W)
    temp = np.array([1.4 ** (i % 50) for i in range(W)])
    for rep in range(3):
        L = -np.abs(rng.normal(0, 50, W))
        idx = rng.permutation(W)
        b = rng.integers(0, W, W)  # includes the void b = W-1 attempts
        beta = rng.uniform(0, 1, W)
        assert np.array_equal(swap_levels(idx, L, temp, b, beta), swap_sequential(idx, L, temp, b, beta))


def test_level_count_is_small():
    """~10 levels at W = 4096: the swap kernel's sequential depth."""
    rng = np.random.default_rng(7)
    lv = levels(rng.integers(0, 4095, 4096), 4096)
    assert lv.max() <= 20


def _seg_lo(lo, nl, g, G):
    return lo + (nl * g) // G


@pytest.mark.parametrize("nl,G,nlv", [(50, 1, 7), (4096, 32, 10), (4096, 32, 0), (1000, 8, 200), (300, 3, 1),
                                      (7, 2, 5), (65536, 512, 14)])
def test_segment_ranges_are_exactly_the_cones(nl, G, nlv):
    """The producer's per-segment attempt lists (hb_dsampler.hip
    pair_segments): for every pair (b, b+1) the returned segments are exactly
    those whose cone [sl - nlv, sh + nlv) holds the pair -- for one process
    and for a rank owning [lo, lo + nl) of a larger ladder."""
    import ctypes as C

    from hb_mcmc_amd import _lib

    lib = _lib.lib()
    g0, g1 = C.c_int(), C.c_int()
    for lo, Wt in ((0, nl), (nl // 3, 3 * nl)):
        sl = np.array([_seg_lo(lo, nl, g, G) for g in range(G + 1)])
        for b in (range(Wt - 1) if Wt <= 5000 else list(range(0, Wt - 1, 5)) + [Wt - 2]):
            want = {g for g in range(G) if sl[g] - nlv <= b and b + 1 < sl[g + 1] + nlv}
            lib.hbx_pair_segments(b, nlv, lo, nl, G, C.byref(g0), C.byref(g1))
            got = set(range(g0.value, g1.value + 1))
            assert want == got, (lo, b, want, got)


def test_device_sampler_symbols_exported():
    from hb_mcmc_amd import _lib, sampler

    lib = sampler._declare(_lib.lib())
    for name in ("hb_dsampler_create", "hb_dsampler_step", "hb_dsampler_download", "hb_mcmc_run_device",
                 "hb_sampler_export", "hb_glibc_eval"):
        assert hasattr(lib, name)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_device_sampler_reproduces_reference_trace(tmp_path):
    from test_sampler import assert_gpu_run_matches_reference, stage_input

    g = stage_input(str(tmp_path))
    exe = os.path.join(ROOT, "hb_mcmc_amd", "lib", "hb_mcmc")
    r = subprocess.run([exe, "1200", "127079833", "0.5021", "0", "--root", str(tmp_path), "--device-sampler"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "device-resident sampler" in r.stdout
    assert_gpu_run_matches_reference(tmp_path, g)


def _host_vs_device(W, niter, ladder, seed_run=0, n=256):
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.dsampler import DeviceSampler
    from hb_mcmc_amd.likelihood import HBLikelihood
    from hb_mcmc_amd.sampler import SlotSampler

    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    s = np.full(n, 1e-3)
    f = truth + s * synth.noise(n)
    L = HBLikelihood(t, f, s)
    L.reserve(W)
    npast = 20
    logp = synth.THETA_STAR[2]
    # host loop with the GPU likelihood
    H = SlotSampler(niter, W, logp, 0, W, run=seed_run, npast=npast, ladder=ladder, nthreads=8)
    x, _, _ = H.get()
    x0 = x.copy()
    H.set_logl(L.loglike(x))
    for it in range(niter):
        y = H.propose(it)
        H.accept(it, L.loglike(y))
        _, ll, _ = H.get()
        perm, _ = H.swap(ll)
        H.apply_perm(perm)
        H.end_iter(it)
    # device loop from a fresh sampler with the same configuration
    D0 = SlotSampler(niter, W, logp, 0, W, run=seed_run, npast=npast, ladder=ladder, nthreads=8)
    with DeviceSampler(D0, L) as D:
        D.init_logl()
        for it in range(niter):
            D.step(it)
        D.download()
    out = []
    for S in (H, D0):
        xs, ls, cid = S.get()
        out.append((xs, ls, cid, S.stats(), S.state_arrays()))
    L.close()
    return out, x0


@pytest.mark.gpu
@pytest.mark.parametrize("W,niter,ladder,n", [(50, 60, 0, 256), (4096, 30, 1, 256), (6000, 24, 1, 256),
                                              (100, 30, 0, 2500), (1000, 40, 1, 1024)])
def test_device_sampler_state_equals_host_sampler(W, niter, ladder, n):
    """n = 2500 takes the multi-wave likelihood plan, where the Hastings test
    runs as its own ds_accept launch instead of the eval kernel's epilogue;
    W = 100 leaves the last workgroup partly filled (36 of 64 slots);
    W = 1000 at n = 1024: 8 swap segments of 125 slots, the records written by
    ds_propose's epilogue."""
    ((hx, hl, hc, hs, ha), (dx, dl, dc, ds, da)), x0 = _host_vs_device(W, niter, ladder, n=n)
    assert np.array_equal(hc, dc), "chain ids by slot"
    assert np.array_equal(hx, dx), "states"
    assert np.array_equal(hl, dl), "logL"
    assert hs == ds, (hs, ds)
    for k in ha:
        assert np.array_equal(ha[k], da[k]), k
    assert hs["nswap"] > 0
    # some proposal was accepted: a final state that no initial state equals
    init = {r.tobytes() for r in x0}
    assert any(r.tobytes() not in init for r in hx), "no proposal accepted: the accept branch never ran"
    if n == 256:  # the sharper 2500-cadence posterior may reject every cold proposal in 30 iterations
        assert hs["cold_acc"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("W", [64, 4096])
def test_deferred_swaps_equal_swap_launches(W, monkeypatch):
    """The tempering swaps deferred into the next ds_propose (HB_DS_DEFER,
    one-slot cone replays, per-slot swap counters, parity-split DE counts)
    against their own ds_swap_seg launch per iteration (HB_DS_DEFER=0): states,
    logL, chain ids and every counter bit for bit, with gathers after
    iterations 0, 7 (odd: the parity-split counters) and 100 (the 100-step
    resets) flushing the pending swaps mid-run, and past NPAST so that
    differential-evolution proposals (chain 0's DE trials) occur."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.dsampler import DeviceSampler
    from hb_mcmc_amd.likelihood import HBLikelihood
    from hb_mcmc_amd.sampler import SlotSampler

    n, niter, npast = 256, 130, 20
    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    s = np.full(n, 1e-3)
    f = truth + s * synth.noise(n)
    runs = []
    for defer in ("1", "0"):
        monkeypatch.setenv("HB_DS_DEFER", defer)
        with HBLikelihood(t, f, s) as L:
            L.reserve(W)
            S = SlotSampler(niter, W, synth.THETA_STAR[2], 0, W, run=3, npast=npast, ladder=1, nthreads=8)
            seen = []
            with DeviceSampler(S, L) as D:
                D.init_logl()
                for it in range(niter):
                    D.step(it)
                    if it in (0, 7, 100):
                        seen.append(D.gather())
                seen.append(D.gather())
                D.download()
            xs, ls, cid = S.get()
            runs.append((seen, xs, ls, cid, S.stats()))
            S.close()
    (sa, xa, la, ca, sta), (sb, xb, lb, cb, stb) = runs
    assert np.array_equal(xa, xb) and np.array_equal(la, lb) and np.array_equal(ca, cb)
    assert sta == stb and sta["nswap"] > 0 and sta["DEtrial"] > 0
    for ga, gb in zip(sa, sb):
        for u, v in zip(ga, gb):
            if isinstance(u, np.ndarray):
                assert np.array_equal(u, v)
            else:
                assert u == v
