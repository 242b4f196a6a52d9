"""Summarise a bench.py JSON line (last line of the file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])


def line(tag, x):
    r = x["roofline"]
    det = x.get("step_ms_detail", {})
    print("%s: value %.4g ms/step %.4f p50 %.4f abi %.4f dev p50 %s kernel %s %.4f ms frac %.3f traffic %s path %s" % (
        tag, x["value"], x["ms_per_step"], x["p50_query_ms"], x.get("p50_c_abi_ms", 0),
        ("%.4f" % det["device_p50"]) if "device_p50" in det else "-", r["kernel"],
        r["kernels"][r["kernel"]]["avg_ms"], r["frac"], r.get("traffic"), x["config"].get("path")))
    print("   steps", {k: (round(v, 4) if isinstance(v, float) else v) for k, v in det.items()})
    if "merge_phases_ms" in x:
        print("   phases", {k: round(v, 3) for k, v in x["merge_phases_ms"].items()})
    if "verify" in x:
        print("   verify", x["verify"].get("match"))
    if "cpu_baseline" in x:
        print("   cpu", x["cpu_baseline"]["value"], x["cpu_baseline"].get("threads"), x["cpu_baseline"].get("host"))


line("config2" if "config4" in d or "k_scan_query" in d["roofline"]["kernels"] else "head", d)
if "config4" in d:
    line("config4", d["config4"])
