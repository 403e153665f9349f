"""Time libhbmi variants (lib/variants/*.so) on the bench workload, each in its
own process, interleaved over rounds (cdna_hip_programming.md rule 24).

    python scripts/ablate.py [bench.py args...]          # likelihood bench
    ABLATE_MODE=sampler python scripts/ablate.py          # device-resident PT-MCMC loop (sampler_rate.py --device)
"""
import glob, json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sorted(glob.glob(os.path.join(ROOT, "hb_mcmc_amd", "lib", "variants", "libhbmi_*.so")))
extra = sys.argv[1:]
mode = os.environ.get("ABLATE_MODE", "bench")
res = {os.path.basename(l): [] for l in libs}
for rnd in range(3):
    for l in libs:
        env = dict(os.environ, HBMI_LIB=l)
        if mode == "sampler":
            cmd = [sys.executable, os.path.join(ROOT, "scripts", "sampler_rate.py"), "--device",
                   "--iters", os.environ.get("ABLATE_STEPS", "200")] + extra
        else:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", os.environ.get("ABLATE_STEPS", "100"),
                   "--warmup", "10", "--no-cpu-baseline"] + extra
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(l, "FAILED", r.stderr[-300:]); continue
        j = json.loads(r.stdout.strip().splitlines()[-1])
        if mode == "sampler":
            res[os.path.basename(l)].append((j["ms_per_iter"], 0.0, j["walkers"] / j["ms_per_iter"] * 1e3))
        else:
            res[os.path.basename(l)].append((j["roofline"]["kernel_ms"], j["roofline"].get("prep_kernel_ms", 0.0),
                                             j["value"]))
for k, v in res.items():
    if v:
        what = "iter_ms" if mode == "sampler" else "eval_ms"
        print(f"{k:28s} {what} min {min(x[0] for x in v):.4f} med {sorted(x[0] for x in v)[len(v)//2]:.4f}  "
              f"prep {min(x[1] for x in v):.4f}  rate/s {max(x[2] for x in v):.3e}")
