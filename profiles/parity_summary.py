"""Regenerate round2_parity_audit/SUMMARY.md from the per-config JSONs that
tests/test_parity_gpu.py writes under RGAN_PARITY_AUDIT=DIR.  usage: python profiles/parity_summary.py DIR"""
import glob
import json
import os
import sys

HEAD = """# GPU step parity audit (round 2, `RGAN_PARITY_AUDIT`, tests/test_parity_gpu.py)

Per config: tensors compared over the teacher-forced iterations, how many met the 1e-4 bar
directly, how many only within 4x the oracle's own fp32-vs-fp64 distance (envelope), and
how many only under the flip rule (downstream of an activation-sign flip, 3e-2).
Each JSON lists every exception by name.

| config | tensors | direct (<= 1e-4) | envelope | flip |
|---|---|---|---|---|
"""


def main(d):
    rows, tot, direct = [], 0, 0
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        r = json.load(open(f))
        assert r.get("FAIL", 0) == 0, f
        rows.append(f"| {r['config']} | {r['tensors']} | {r['direct']} | {r['envelope']} | {r['flip']} |")
        tot += r["tensors"]
        direct += r["direct"]
    out = HEAD + "\n".join(rows) + f"\n\nTotal: {direct} of {tot} tensors direct ({100.0 * direct / tot:.1f} %).\n"
    open(os.path.join(d, "SUMMARY.md"), "w").write(out)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1])
