"""Probe the GPU box's host CPU share: thread scaling of the reference batch."""
import os, sys, time, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
from hb_mcmc_amd import synth
import oracle as orc
print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count(), "OMP", os.environ.get("OMP_NUM_THREADS"))
for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu.weight"):
    try: print(p, open(p).read().strip())
    except Exception as e: print(p, e)
print(subprocess.run("lscpu | grep -E 'Model name|^CPU\\(s\\)|Thread|MHz'", shell=True, capture_output=True, text=True).stdout)
impl = orc.Reference() if orc.reference_available() else orc.Oracle()
t, f, s = synth.dataset(1024, impl.light_curve)
P = synth.walkers(2000, seed=4243)
for nt in (1, 1, 2, 4, 8, 16, 16, 32):
    w = min(len(P), 120 * nt)
    t0 = time.perf_counter(); impl.loglike_batch(t, f, s, P[:w], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, nt)
    print(nt, w, round(w / (time.perf_counter() - t0)))
