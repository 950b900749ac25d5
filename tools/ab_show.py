import glob, json, sys
for f in sorted(glob.glob("gpurun_out/ab_%s_*.log" % sys.argv[1])):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no result"); continue
    d = json.loads(lines[-1])
    print("%-45s step %.4f ms  scan %.4f  feed %.4f  distinct %d  frac %.3f" % (
        f, d["ms_per_step"], d["scan_kernel_ms"], d["feed_device_ms"], d["distinct_kmers"], d["roofline"]["frac"]))
