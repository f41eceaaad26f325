"""Effective shader clock per dispatch of the tracer kernel (GRBM_GUI_ACTIVE / 8 XCDs / kernel
time): run a render_once command under rocprofv3 --pmc GRBM_GUI_ACTIVE, then
  python tools/clock_check.py PMC_DIR RENDER_ONCE_LOG
prints, frame by frame, the kernel ms (HIP events) and the clock."""
import csv
import json
import sys

pmc_dir, log = sys.argv[1], sys.argv[2]
rows = [r for r in csv.DictReader(open(f"{pmc_dir}/run_counter_collection.csv"))
        if r["Kernel_Name"].startswith("vcrt_trace") and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
st = None
for line in open(log):
    if line.startswith("[") or line.startswith("{"):
        st = json.loads(line)
st = st if isinstance(st, list) else [st]
for i, (r, s) in enumerate(zip(rows, st)):
    ms = s["kernel_ms"]
    print(f"frame {i}: {ms:.3f} ms, clock {float(r['Counter_Value']) / 8 / (ms * 1e-3) / 1e9:.3f} GHz")
