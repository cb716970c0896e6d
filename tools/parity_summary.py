"""Summarise a GPU parity audit (RGAN_PARITY_AUDIT=dir of tests/test_parity_gpu.py) into the
committed forms: <out_dir>/SUMMARY.md (the per-config table) and <summary.json> (the compact
record bench.py's emu_parity_evidence reads).

usage: python tools/parity_summary.py AUDIT_DIR OUT_DIR SUMMARY_JSON "head / run note"
"""
import glob
import json
import os
import shutil
import sys

HEADER = """# GPU step parity audit ({round}, `RGAN_PARITY_AUDIT`, tests/test_parity_gpu.py, head {head})

Per config: tensors compared over the teacher-forced iterations and how each met its
tolerance (1e-4 outputs / losses / GP and buffers, 2e-4 gradients):
  * direct   -- GPU vs the fp32 oracle (pinned bitwise to the reference);
  * forced   -- GPU vs the same step in float64 with every ReLU / LeakyReLU / SELU taking the
                GPU's branch (the mask-forced judge: what remains is arithmetic, not which side
                of a kink a value within rounding of 0 fell on);
  * envelope -- within 4x the oracle's own fp32-vs-fp64 distance (biases feeding BatchNorm:
                exact gradient 0);
  * flip     -- downstream of an activation-sign flip, 3e-2 (unused).
The forced judge proves its premise: `sign flips` counts the GPU activation signs that differ
from the exact step's, and `max |x|/RMS at a flip` is the largest exact pre-activation at any
of them relative to that activation call's RMS (must be <= TAU_FLIP = 1e-4).  Outputs and
gradients also pass elementwise against the forced step: `worst elem` = max over tensors of
max|gpu - forced| / (RMS(forced) * tol) (must be <= ELEM_FACTOR = 10).
`-bf16x6` rows: the same configs with the opt-in fp32-on-bf16x6 forward / data-gradient GEMMs
(`-m gpu_emu`).

| config | tensors | direct | forced | direct or forced | envelope | flip | sign flips | max \\|x\\|/RMS at a flip | worst elem (x tol) |
|---|---|---|---|---|---|---|---|---|---|
"""


def main():
    audit, out_dir, out_json, head = sys.argv[1:5]
    rnd = os.path.basename(out_dir.rstrip("/")).replace("_parity_audit", "").replace("round", "round ")
    os.makedirs(out_dir, exist_ok=True)
    rows, compact = [], {}
    tot = {"tensors": 0, "direct": 0, "forced": 0, "envelope": 0, "flip": 0, "FAIL": 0}
    for f in sorted(glob.glob(os.path.join(audit, "*.json"))):
        d = json.load(open(f))
        if "tensors" not in d:  # the drift record and other non-step audits travel as they are
            shutil.copy(f, out_dir)
            continue
        name = d["config"]
        shutil.copy(f, out_dir)
        nflip = sum(e.get("elements", 1) for e in d.get("flips", []))
        w = d.get("worst_elem_vs_forced") or {}
        welem = (w["max_over_rms"] / w["tol"]) if w else 0.0
        prem = d.get("premise_max_abs_over_rms", 0.0)
        rows.append(f"| {name} | {d['tensors']} | {d['direct']} | {d['forced']} | {d['direct'] + d['forced']} | "
                    f"{d['envelope']} | {d['flip']} | {nflip} | {('%.2e' % prem) if nflip else '-'} | {welem:.2f} |")
        compact[name] = {k: d[k] for k in ("tensors", "direct", "forced", "envelope", "flip", "FAIL")}
        compact[name]["premise_max_abs_over_rms"] = prem
        compact[name]["worst_elem_vs_forced"] = w
        for k in tot:
            tot[k] += d[k] or 0
    with open(os.path.join(out_dir, "SUMMARY.md"), "w") as fh:
        fh.write(HEADER.format(round=rnd, head=head))
        fh.write("\n".join(rows) + "\n")
        fh.write(f"\nTotal: {tot['tensors']} tensors, {tot['direct']} direct, {tot['forced']} forced "
                 f"({tot['direct'] + tot['forced']} direct or forced), {tot['envelope']} envelope, "
                 f"{tot['flip']} flip, {tot['FAIL']} failed.\n")
    with open(out_json, "w") as fh:
        json.dump({"audit": os.path.basename(out_dir.rstrip("/")), "head": head, "configs": compact, "total": tot},
                  fh, indent=1)
    print(f"{len(compact)} configs, {tot}")


if __name__ == "__main__":
    main()
