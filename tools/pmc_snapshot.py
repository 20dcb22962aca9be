"""SnapshotV1 kernels' rocprofv3 counters -> profiles/r<NN>_pmc_snapshot_config5_<docs>docs.json.

Input: the counter_collection CSVs of separate `rocprofv3 --pmc ...` passes over the same
`bench.py --config 5 --docs D --steps 1 --warmup 0 --no-cpu` command (scripts/r4_prof.sh pmcA5 /
pmcB5 / pmcw5).  Counters are summed over the step's dispatches of each snapshot kernel (one per
replay launch) and over their instances.  Derived per kernel: instructions and wave cycles per
document, the share of wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES), and the bytes
written to HBM (WRITE_SIZE is in KiB) against the JSON bytes the step produced.

usage: python tools/pmc_snapshot.py --docs D --json-bytes B --out OUT CSV [CSV ...]
"""
import argparse
import collections
import csv
import json

KERNELS = ("mt_snapshot_kernel", "mt_snapshot_size_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, required=True)
    ap.add_argument("--json-bytes", type=int, required=True, help="SnapshotV1 bytes of the step")
    ap.add_argument("--out", required=True)
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args()
    acc = collections.defaultdict(float)
    for p in a.csv:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if k in KERNELS:
                acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    out = {"command": f"bench.py --config 5 --docs {a.docs} --steps 1 --warmup 0 --no-cpu",
           "units": "counters summed over the step's dispatches of each kernel and over instances",
           "json_bytes": a.json_bytes, "kernels": {}}
    for k in KERNELS:
        c = {n: v for (kk, n), v in sorted(acc.items()) if kk == k}
        if not c:
            continue
        d = {"counters": c}
        ins = sum(c.get(n, 0.0) for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS",
                                          "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"))
        if "SQ_INSTS_VALU" in c:
            d["instructions_per_doc"] = round(ins / a.docs)
        if "SQ_WAVE_CYCLES" in c:
            d["wave_cycles_per_doc"] = round(c["SQ_WAVE_CYCLES"] * 4 / a.docs)
            if "SQ_WAIT_ANY" in c:
                d["wait_share"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
        if "WRITE_SIZE" in c:
            d["hbm_write_bytes"] = int(c["WRITE_SIZE"] * 1024)
            if k == "mt_snapshot_kernel":
                d["write_bytes_over_json_bytes"] = round(c["WRITE_SIZE"] * 1024 / a.json_bytes, 3)
        out["kernels"][k] = d
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: {x: y for x, y in v.items() if x != "counters"} for k, v in out["kernels"].items()}))


if __name__ == "__main__":
    main()
