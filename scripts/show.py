import glob, json, sys
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/bench_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1]); r = d["roofline"]
        print(f"{f.split('/')[-1]:28s} {d['value']:.3g} gs/s  ms/step {d['ms_per_step']:.4f}  kern {r['kernel_avg_ms']:.3f} ms/launch  frac {r['frac']:.3f} valid={d['valid']}")
    except Exception as ex:
        print(f, "ERR", ex)
