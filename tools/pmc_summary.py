"""Summarise rocprofv3 PMC passes (tools/profile.sh output) per kernel:
mean counter value per dispatch of encode_kernel / decode_kernel, plus the
HBM-traffic fields bench.py reads (FETCH_SIZE doubled on gfx950 and
WRITE_SIZE, both in KB per rocprofv3 -> bytes).
usage: python tools/pmc_summary.py gpurun_out/<tag> [--json out.json WORKLOAD] (merged by WORKLOAD)
(WORKLOAD: the bench config string the passes ran, stored with the numbers so
bench.py only reports traffic measured on its own workload)"""
import csv
import re
import json
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(root.glob("*/*_counter_collection.csv")):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"]
            short = ("e4_size_kernel" if "e4_size_kernel" in k else "e4_emit_kernel" if "e4_emit_kernel" in k
                     else "sp_encode_sparse_kernel" if "cpk_sparse" in k and "sp_encode_kernel" in k
                     else "sp_encode_kernel" if "sp_encode_kernel" in k
                     else "decode2_kernel" if "decode2_kernel" in k
                     # (decode_kernel<stream, serial>: the dense form -- serial walks of
                     # dense windows -- is its own launch, skipped unless picked)
                     else "decode_kernel_dense" if re.search(r"decode_kernel<\w+, ?true>", k)
                     else "decode_kernel" if "decode_kernel" in k else k.split("(")[0][-40:])
            vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for kern in ("sp_encode_kernel", "sp_encode_sparse_kernel", "e4_size_kernel", "e4_emit_kernel", "decode_kernel",
             "decode_kernel_dense", "decode2_kernel"):
    if kern not in vals:
        continue
    d = {c: sum(v) / len(v) for c, v in vals[kern].items()}
    out[kern] = d
    print(kern)
    for c in sorted(d):
        print(f"  {c:24s} {d[c]:18.1f}")
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        print(f"  VALU instr / wave      {d['SQ_INSTS_VALU'] / d['SQ_WAVES']:.0f}")
        print(f"  SALU instr / wave      {d['SQ_INSTS_SALU'] / d['SQ_WAVES']:.0f}")
        print(f"  LDS  instr / wave      {d['SQ_INSTS_LDS'] / d['SQ_WAVES']:.0f}")
    if "SQ_WAVE_CYCLES" in d:
        wc = d["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in d:
                print(f"  {c:22s} {100 * d[c] / wc:6.1f} % of wave cycles")
if len(sys.argv) > 3 and sys.argv[2] == "--json":
    traffic = {}
    # The library enqueues both encoders (and both batch decoders) and the
    # one not chosen returns at once: the stage's traffic is the working
    # one's -- the larger (the v4 encode stage = size pass + emit pass)
    def traffic_of(d):
        return d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)
    enc = []
    for k in ("sp_encode_kernel", "sp_encode_sparse_kernel"):
        if k in out:
            enc.append(out[k])
    if "e4_size_kernel" in out and "e4_emit_kernel" in out:
        enc.append({c: out["e4_size_kernel"].get(c, 0) + out["e4_emit_kernel"].get(c, 0)
                    for c in ("FETCH_SIZE", "WRITE_SIZE")})
    if enc:
        out["encode_kernel"] = max(enc, key=traffic_of)
    dec = [out[k] for k in ("decode_kernel", "decode_kernel_dense", "decode2_kernel") if k in out]
    if dec:
        out["decode_kernel"] = max(dec, key=traffic_of)
    for kern, key in (("encode_kernel", "encode"), ("decode_kernel", "decode")):
        d = out.get(kern, {})
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            # rocprofv3 reports KB; gfx950 FETCH_SIZE counts half the bytes of
            # wide streaming reads (MI355X_MICROARCH.md HBM section)
            traffic[key] = {"fetch_bytes": 2 * 1024 * d["FETCH_SIZE"], "write_bytes": 1024 * d["WRITE_SIZE"],
                            "hbm_bytes": 2 * 1024 * d["FETCH_SIZE"] + 1024 * d["WRITE_SIZE"]}
    traffic["source"] = str(root)
    # one entry per workload in the file (merged with what it holds)
    key = sys.argv[4] if len(sys.argv) > 4 else "unknown"
    dst = Path(sys.argv[3])
    try:
        allw = json.loads(dst.read_text()) if dst.exists() else {}
        if "workload" in allw:  # (the single-workload form of round 1)
            allw = {}
    except ValueError:
        allw = {}
    allw[key] = traffic
    dst.write_text(json.dumps(allw, indent=1, sort_keys=True))
    print(json.dumps(traffic))
