"""Fold a tools/r04_pmc.sh output tree into profiles/valu.json and
profiles/traffic.json: per (kernel, nodes, config) the mean per dispatch of
SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES / SQ_WAVE_CYCLES / SQ_ACTIVE_INST_VALU
/ SQ_WAIT_ANY / SQ_WAIT_INST_ANY (summed over XCD / SE instances of one
dispatch) and HBM bytes = 2 x FETCH_SIZE KiB + WRITE_SIZE KiB (gfx950
corrections, MI355X_MICROARCH.md HBM section).
On the box (r04_pmc.sh): python3 tools/pmc_entries.py gpurun_out/<tag> --box writes <tag>/entries.json;
here: python3 tools/pmc_entries.py gpurun_out/<tag> profiles/r04/pmc folds entries.json into profiles/."""
import collections
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC, KEEP = sys.argv[1], sys.argv[2]
# config label -> (bench config, nodes)
CFG = {"c1": (1, 5000), "c1a": (1, 5000), "c2": (2, 5000), "c2a": (2, 5000), "c3": (3, 10000), "c4": (4, 100000), "c4a": (4, 100000),
       "c5": (5, 5000)}
# kernel symbol -> the bench kernel table's slot name
NAME = {"k_adapt_mask_ns": "k_adapt_mask"}
# kernels launched together in one slot (the doubling ADAPT window): per batch,
# the sum over the group's dispatches; the anchor runs once per batch
GROUP = {"k_win_build": "k_adapt_window", "k_win_round": "k_adapt_window", "k_win_final": "k_adapt_window"}
ANCHOR = {"k_adapt_window": "k_win_final"}


def kname(raw):
    k = raw.split("(")[0].split("<")[0].replace("void ", "").replace("ksim::", "").strip()
    return NAME.get(k, k)


if KEEP != "--box" and os.path.exists(os.path.join(SRC, "entries.json")):
    new_v, new_t = json.load(open(os.path.join(SRC, "entries.json")))
    valu = json.load(open(os.path.join(ROOT, "profiles", "valu.json")))
    traffic = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
    key = lambda e: (e.get("kernel"), e.get("nodes"), e.get("config"))
    for lst, new in ((valu, new_v), (traffic, new_t)):
        ks = {key(e) for e in new}
        lst[:] = [e for e in lst if key(e) not in ks] + [dict(e, source=e["source"].replace("<KEEP>", KEEP))
                                                         for e in new]
    json.dump(valu, open(os.path.join(ROOT, "profiles", "valu.json"), "w"), indent=1)
    json.dump(traffic, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    os.makedirs(os.path.join(ROOT, KEEP), exist_ok=True)
    for f in ("summary.txt", "entries.json"):
        shutil.copy(os.path.join(SRC, f), os.path.join(ROOT, KEEP, f))
    print([key(e) for e in new_v])
    sys.exit(0)
per = collections.defaultdict(float)
for f in glob.glob(os.path.join(SRC, "*", "**", "*counter_collection.csv"), recursive=True):
    label = os.path.relpath(f, SRC).split(os.sep)[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(f)):
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[(label, kname(r["Kernel_Name"]), r["Counter_Name"], d)] += float(r["Counter_Value"])
acc = collections.defaultdict(list)
gsum, gcnt = collections.defaultdict(float), collections.defaultdict(int)
for (label, k, c, _), v in per.items():
    if k in GROUP:
        slot = GROUP[k]
        gsum[(label, slot, c)] += v
        gcnt[(label, slot, c)] += k == ANCHOR[slot]
        continue
    acc[(label, k, c)].append(v)
mean = {key: statistics.mean(v) for key, v in acc.items()}
mean.update({key: v / gcnt[key] for key, v in gsum.items() if gcnt[key]})
valu, traffic = [], []
src = f"<KEEP>/summary.txt (tools/r04_pmc.sh + tools/pmc_entries.py: rocprofv3 --pmc, one pass per counter group, " \
      "kernel trace only; counters summed over XCD/SE instances per dispatch, averaged over dispatches; " \
      "HBM bytes = 2 x FETCH_SIZE KiB + WRITE_SIZE KiB)"
done = []
for (label, k, c), v in sorted(mean.items()):
    if c != "SQ_INSTS_VALU" or label not in CFG:
        continue
    cfg, nodes = CFG[label]
    g = lambda name: mean.get((label, k, name))
    ve = {"kernel": k, "nodes": nodes, "config": cfg, "mode": "adapt" if label.endswith("a") and label != "c5" else "p100",
          "valu_insts_per_launch": v, "salu_insts_per_launch": g("SQ_INSTS_SALU"),
          "waves_per_launch": g("SQ_WAVES"), "wave_quad_cycles_per_launch": g("SQ_WAVE_CYCLES"),
          "valu_active_quad_cycles_per_launch": g("SQ_ACTIVE_INST_VALU"),
          "wait_any_quad_cycles_per_launch": g("SQ_WAIT_ANY"),
          "wait_inst_any_quad_cycles_per_launch": g("SQ_WAIT_INST_ANY"), "source": src + f" [{label}]"}
    valu = [e for e in valu if not (e.get("kernel") == k and e.get("nodes") == nodes and e.get("config") == cfg)]
    valu.append(ve)
    fetch = mean.get((label, k, "FETCH_SIZE"))
    write = mean.get((label, k, "WRITE_SIZE"))
    if fetch is not None and write is not None:
        te = {"kernel": k, "nodes": nodes, "config": cfg, "hbm_bytes_per_launch": 2 * fetch * 1024 + write * 1024,
              "hbm_read_bytes_per_launch": 2 * fetch * 1024, "hbm_write_bytes_per_launch": write * 1024,
              "source": src + f" [{label}]"}
        traffic = [e for e in traffic if not (e.get("kernel") == k and e.get("nodes") == nodes and e.get("config") == cfg)]
        traffic.append(te)
    done.append((label, k))
json.dump([valu, traffic], open(os.path.join(SRC, "entries.json"), "w"), indent=1)
print(done)
