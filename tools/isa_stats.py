"""Instruction mix of kernels in a hipcc -S device assembly file, per basic block loop.
usage: python tools/isa_stats.py FILE.s SUBSTRING [--loops]"""
import re
import sys

src = open(sys.argv[1]).read()
want = sys.argv[2]
for m in re.finditer(r"^(_ZN4rgan\S+):", src, re.M):
    name = m.group(1)
    if want not in name:
        continue
    end = src.find(".Lfunc_end", m.end())
    body = src[m.end():end]
    ins = [l.split(";")[0].strip() for l in body.split("\n")]
    ins = [l for l in ins if l and not l.startswith((".", ";", "//"))]
    cnt = {}
    for l in ins:
        if l.endswith(":"):
            continue
        op = l.split()[0]
        k = ("mfma" if op.startswith("v_mfma") else "ds_read" if op.startswith("ds_read") else
             "ds_write" if op.startswith("ds_write") else "vmem" if op.startswith(("global_", "buffer_")) else
             "waitcnt" if op.startswith("s_waitcnt") else "barrier" if op == "s_barrier" else
             "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else op)
        cnt[k] = cnt.get(k, 0) + 1
    print(name[:80], dict(sorted(cnt.items())))
    if "--loops" in sys.argv:
        # basic blocks that are loop targets (branch back): print their mix
        labels = {}
        cur = None
        for l in ins:
            if l.endswith(":"):
                cur = l[:-1]
                labels[cur] = []
                continue
            if cur:
                labels[cur].append(l)
        for lab, lines in labels.items():
            ops = [x.split()[0] for x in lines]
            if any(x.startswith("s_cbranch") and lab in y for x, y in zip(ops, lines)):
                mf = sum(o.startswith("v_mfma") for o in ops)
                print(f"  loop {lab}: {len(ops)} ins, mfma {mf}, ds_read {sum(o.startswith('ds_read') for o in ops)}, "
                      f"ds_write {sum(o.startswith('ds_write') for o in ops)}, waitcnt {sum(o.startswith('s_waitcnt') for o in ops)}, "
                      f"valu {sum(o.startswith('v_') and not o.startswith('v_mfma') for o in ops)}, "
                      f"vmem {sum(o.startswith(('global_', 'buffer_')) for o in ops)}, barrier {ops.count('s_barrier')}")
