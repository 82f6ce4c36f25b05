"""Print an r3_ab.sh / r3_modes.sh run: per-kernel extraction times (new vs old) and the bench values."""
import glob
import json
import re
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "ab"
for f in sorted(glob.glob(f"gpurun_out/{tag}_x*.log")):
    txt = open(f).read()
    ks = dict(re.findall(r"^\s+(k_\w+)\s+([\d.]+) us/call", txt, re.M))
    tot = re.search(r"extract: ([\d.]+) us", txt)
    print(f.split("/")[-1], tot.group(1) if tot else "?", " ".join(f"{k}={v}" for k, v in sorted(ks.items())))
for f in sorted(glob.glob(f"gpurun_out/{tag}_b*.log") + glob.glob(f"gpurun_out/{tag}_m*.log")
                + glob.glob(f"gpurun_out/{tag}_parity.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split("/")[-1], d["value"], d.get("parity_bit_exact", ""),
              {k: v for k, v in d["kernels_us_per_subbatch"].items()})
    except Exception as e:  # noqa: BLE001
        print(f, "failed", e)
