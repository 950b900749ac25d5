import csv, glob, sys
kern = sys.argv[2] if len(sys.argv) > 2 else "scan_planes"
for d in sorted(glob.glob("gpurun_out/pmc_%s_*/" % sys.argv[1])):
    fs = glob.glob(d + "*counter_collection.csv")
    if not fs:
        print(d, "none"); continue
    agg = {}
    for r in csv.DictReader(open(fs[0])):
        if kern in r["Kernel_Name"]:
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    w = m.get("SQ_WAVES", 1)
    print("%-32s waves %.0f VALU/w %.1f SALU/w %.1f LDS/w %.1f VMEM/w %.2f SMEM/w %.2f busy %.3g" % (
        d, w, m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_SALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w,
        m.get("SQ_INSTS_VMEM_RD", 0) / w, m.get("SQ_INSTS_SMEM", 0) / w, m.get("SQ_BUSY_CYCLES", 0)))
