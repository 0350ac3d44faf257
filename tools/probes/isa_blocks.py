"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (VALU / MFMA / LDS /
global / scalar / waits), to find where a kernel's issue slots go.
usage: python tools/probes/isa_blocks.py file.s <kernel-name-substring> [min_instructions]"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name) or (re.match(r"^_Z\S+:", l) and name in l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks, cur, label = [], [], "entry"
    for l in lines[start + 1:end]:
        s = l.strip()
        if re.match(r"^\.LBB\S+:", s):
            blocks.append((label, cur))
            label, cur = s.split(":")[0] + ("  " + s.split(";")[1].strip() if ";" in s else ""), []
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.append(s.split()[0])
    blocks.append((label, cur))
    tot = {}
    for label, ins in blocks:
        c = dict(mfma=0, valu=0, ds_r=0, ds_w=0, glob=0, salu=0, wait=0, branch=0, other=0)
        for op in ins:
            if op.startswith("v_mfma"):
                c["mfma"] += 1
            elif op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("ds_read") or op.startswith("ds_load"):
                c["ds_r"] += 1
            elif op.startswith("ds_"):
                c["ds_w"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["glob"] += 1
            elif op.startswith("s_waitcnt") or op.startswith("s_barrier"):
                c["wait"] += 1
            elif op.startswith(("s_cbranch", "s_branch")):
                c["branch"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            else:
                c["other"] += 1
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        if len(ins) >= mn:
            print(f"{label[:60]:60s} n={len(ins):5d} " + " ".join(f"{k}={v}" for k, v in c.items() if v))
    print("TOTAL", " ".join(f"{k}={v}" for k, v in tot.items()))


if __name__ == "__main__":
    main()
