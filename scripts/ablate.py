"""Time libhbmi variants (lib/variants/*.so) on the bench workload, each in its
own process, interleaved over rounds (cdna_hip_programming.md rule 24)."""
import glob, json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sorted(glob.glob(os.path.join(ROOT, "hb_mcmc_amd", "lib", "variants", "libhbmi_*.so")))
extra = sys.argv[1:]
res = {os.path.basename(l): [] for l in libs}
for rnd in range(3):
    for l in libs:
        env = dict(os.environ, HBMI_LIB=l)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", os.environ.get("ABLATE_STEPS", "100"), "--warmup", "10",
                            "--no-cpu-baseline"] + extra, env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(l, "FAILED", r.stderr[-300:]); continue
        j = json.loads(r.stdout.strip().splitlines()[-1])
        res[os.path.basename(l)].append((j["roofline"]["kernel_ms"], j["roofline"]["prep_kernel_ms"], j["value"]))
for k, v in res.items():
    if v:
        print(f"{k:28s} eval_ms min {min(x[0] for x in v):.4f} med {sorted(x[0] for x in v)[len(v)//2]:.4f}  "
              f"prep {min(x[1] for x in v):.4f}  evals/s {max(x[2] for x in v):.3e}")
