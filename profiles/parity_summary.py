"""Regenerate <DIR>/SUMMARY.md from the per-config JSONs that tests/test_parity_gpu.py
writes under RGAN_PARITY_AUDIT=DIR.  usage: python profiles/parity_summary.py DIR [head] [round]"""
import glob
import json
import os
import sys

HEAD = """# GPU step parity audit (round {rnd}, `RGAN_PARITY_AUDIT`, tests/test_parity_gpu.py{head})

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
`-bf16x6` rows: the same configs with the opt-in fp32-on-bf16x6 forward / data-gradient GEMMs.

| config | tensors | direct | forced | direct or forced | envelope | flip | sign flips | max \\|x\\|/RMS at a flip | worst elem (x tol) |
|---|---|---|---|---|---|---|---|---|---|
"""


def main(d, head="", rnd="4"):
    rows, tot, direct, forced = [], 0, 0, 0
    compact = {}
    drift = []
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        r = json.load(open(f))
        if os.path.basename(f).startswith("drift_"):  # tests/test_drift_gpu.py: a trajectory report
            worst = max(v["max_gap_over_bound"] for v in r["report"].values())
            mean = max(v["gpu_mean_gap"] / v["ref_mean_spread"] for v in r["report"].values() if v["ref_mean_spread"])
            drift.append(f"| {os.path.basename(f)[6:-5]} | {len(r['gpu'].get('errD', r['gpu']))} | "
                         f"{r.get('threads', '-')} | {worst:.2f} | {mean:.2f} |")
            continue
        assert r.get("FAIL", 0) == 0, f
        compact[r["config"]] = {k: r.get(k) for k in ("tensors", "direct", "forced", "envelope", "flip", "FAIL",
                                                      "premise_max_abs_over_rms", "worst_elem_vs_forced")}
        fl = sum(x["elements"] for x in r.get("flips", []))
        we = r.get("worst_elem_vs_forced")
        wtxt = f"{we['max_over_rms'] / we['tol']:.2f}" if we else "-"
        prem = r.get("premise_max_abs_over_rms")
        ptxt = f"{prem:.2e}" if prem else "-"
        rows.append(f"| {r['config']} | {r['tensors']} | {r['direct']} | {r.get('forced', 0)} | "
                    f"{r['direct'] + r.get('forced', 0)} | {r['envelope']} | {r['flip']} | {fl} | {ptxt} | {wtxt} |")
        tot += r["tensors"]
        direct += r["direct"]
        forced += r.get("forced", 0)
    out = (HEAD.format(rnd=rnd, head=f", head {head}" if head else "") + "\n".join(rows) +
           f"\n\nTotal: {direct} of {tot} tensors direct ({100.0 * direct / tot:.1f} %), "
           f"{direct + forced} direct or against the mask-forced fp64 step ({100.0 * (direct + forced) / tot:.1f} %).\n")
    if drift:
        out += ("\nTrajectories vs the reference's thread envelope (tests/test_drift_gpu.py; bound: "
                "3 x the 2-step-lagged spread of the reference's thread-count runs + 1e-4 scale, per step;"
                " mean gap <= the mean spread):\n\n| config | iterations | reference threads | worst step "
                "gap / bound | worst mean gap / mean spread |\n|---|---|---|---|---|\n" + "\n".join(drift) + "\n")
    open(os.path.join(d, "SUMMARY.md"), "w").write(out)
    # compact per-config counts (read by bench.py on the GPU box, where the audit dir is not sent)
    with open(os.path.join(os.path.dirname(os.path.abspath(d)), f"round{rnd}_parity_summary.json"), "w") as fh:
        json.dump({"audit": os.path.basename(os.path.abspath(d)), "head": head, "configs": compact}, fh, indent=1)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "", sys.argv[3] if len(sys.argv) > 3 else "4")
