"""Regenerate <DIR>/SUMMARY.md from the per-config JSONs that tests/test_parity_gpu.py
writes under RGAN_PARITY_AUDIT=DIR.  usage: python profiles/parity_summary.py DIR [head]"""
import glob
import json
import os
import sys

HEAD = """# GPU step parity audit (round 3, `RGAN_PARITY_AUDIT`, tests/test_parity_gpu.py{head})

Per config: tensors compared over the teacher-forced iterations and how each met its
tolerance (1e-4 outputs / losses / GP and buffers, 2e-4 gradients):
  * direct   -- GPU vs the fp32 oracle (pinned bitwise to the reference);
  * forced   -- GPU vs the same step in float64 with every ReLU / LeakyReLU / SELU taking the
                GPU's branch (the mask-forced judge: what remains is arithmetic, not which side
                of a kink a value within rounding of 0 fell on);
  * envelope -- within 4x the oracle's own fp32-vs-fp64 distance;
  * flip     -- downstream of an activation-sign flip, 3e-2.
Each JSON lists every tensor with its errors; `flips` counts the sign disagreements.

| config | tensors | direct | forced | direct or forced | envelope | flip | sign flips |
|---|---|---|---|---|---|---|---|
"""


def main(d, head=""):
    rows, tot, direct, forced = [], 0, 0, 0
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        r = json.load(open(f))
        assert r.get("FAIL", 0) == 0, f
        fl = sum(x["elements"] for x in r.get("flips", []))
        rows.append(f"| {r['config']} | {r['tensors']} | {r['direct']} | {r.get('forced', 0)} | "
                    f"{r['direct'] + r.get('forced', 0)} | {r['envelope']} | {r['flip']} | {fl} |")
        tot += r["tensors"]
        direct += r["direct"]
        forced += r.get("forced", 0)
    out = (HEAD.format(head=f", head {head}" if head else "") + "\n".join(rows) +
           f"\n\nTotal: {direct} of {tot} tensors direct ({100.0 * direct / tot:.1f} %), "
           f"{direct + forced} direct or against the mask-forced fp64 step ({100.0 * (direct + forced) / tot:.1f} %).\n")
    open(os.path.join(d, "SUMMARY.md"), "w").write(out)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
