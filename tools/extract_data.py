"""Extract the reference's DATA files the simulator counterpart reads.

Run once in the build container (the reference tree is not on the GPU box):

    python tools/extract_data.py

Writes
  data/v100_throughputs.json   isolated single-job v100 throughputs (steps/s),
                               the "null" entries of
                               scheduler/shockwave_wisr_throughputs.json, keyed
                               "<job_type>|<scale_factor>"
  data/traces/*.trace          the Shockwave traces, byte for byte
                               (scheduler/traces/shockwave/*.trace)
  data/configs/*.json          the Shockwave policy configs
                               (scheduler/shockwave_replicate/scale_*gpus.json)

These are data (trace rows and measured throughputs), not reference source.
"""
import ast
import json
import os
import shutil

REF = "/root/reference/scheduler"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    raw = json.load(open(os.path.join(REF, "shockwave_wisr_throughputs.json")))
    out = {}
    for key, row in raw["v100"].items():
        job_type, sf = ast.literal_eval(key)
        out[f"{job_type}|{sf}"] = row["null"]
    os.makedirs(os.path.join(ROOT, "data", "traces"), exist_ok=True)
    with open(os.path.join(ROOT, "data", "v100_throughputs.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    src = os.path.join(REF, "traces", "shockwave")
    for name in sorted(os.listdir(src)):
        if name.endswith(".trace"):
            shutil.copyfile(os.path.join(src, name), os.path.join(ROOT, "data", "traces", name))
    os.makedirs(os.path.join(ROOT, "data", "configs"), exist_ok=True)
    cfg = os.path.join(REF, "shockwave_replicate")
    for name in sorted(os.listdir(cfg)):
        if name.startswith("scale_") and name.endswith(".json"):
            shutil.copyfile(os.path.join(cfg, name), os.path.join(ROOT, "data", "configs", name))
    print(f"{len(out)} throughputs, traces: {sorted(os.listdir(os.path.join(ROOT, 'data', 'traces')))}")


if __name__ == "__main__":
    main()
