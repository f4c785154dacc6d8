"""profiles/traffic.json from one measurement session's PMC summaries.

Usage: python tools/make_traffic.py TAG PREFIX
Reads gpurun_out/TAG_<w>pmc_p*/ (tools/r03_measure.sh) through
tools/pmc_traffic.py's corrections for every workload w, writes
gpurun_out/TAG_<w>_pmc.json and gpurun_out/TAG_traffic.json; the latter is
committed as profiles/traffic.json, with the per-workload summaries under
profiles/<PREFIX>_<w>_pmc.json, which each entry names.  bench.py picks the
entry by workload name (never by file order)."""
import json
import os
import subprocess
import sys

tag, prefix = sys.argv[1], sys.argv[2]
here = os.path.dirname(os.path.abspath(__file__))
out = {}
for w in ("c2", "c3", "c4", "c5", "c6", "c7"):
    if not os.path.isdir(f"gpurun_out/{tag}_{w}pmc_p1"):
        continue
    dst = f"gpurun_out/{tag}_{w}_pmc.json"
    subprocess.run([sys.executable, os.path.join(here, "pmc_traffic.py"), f"{tag}_{w}pmc", dst, "resample_"], check=True,
                   stdout=subprocess.DEVNULL)
    rec = json.load(open(dst))
    if "hbm_bytes_per_launch" not in rec:
        continue
    out[w] = {"file": f"profiles/{prefix}_{w}_pmc.json", "session": tag,
              "hbm_bytes_per_launch": int(rec["hbm_bytes_per_launch"]),
              "hbm_read_bytes_per_launch": int(rec["hbm_read_bytes_per_launch"]),
              "hbm_write_bytes_per_launch": int(rec["hbm_write_bytes_per_launch"]),
              "correction": rec["correction"]}
json.dump(out, open(f"gpurun_out/{tag}_traffic.json", "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1))
