"""Static instruction counts of one kernel in a gfx950 assembly file
(hipcc --cuda-device-only -S).  Usage: isa_stats.py FILE.s [FILE2.s ...] [--kernel SUBSTR]

Prints, per file, the kernel's total / VALU / SALU / memory instruction counts and
its register usage (a quick A/B of a source change before a GPU run)."""
import argparse
import re


def kernel_body(text, sym):
    i = text.index("\n" + sym + ":") + 1
    j = text.index(".Lfunc_end", i)   # the whole function (a kernel may have several s_endpgm)
    return text[i:j]


def stats(path, substr):
    text = open(path).read()
    syms = [s for s in re.findall(r"^(_Z[A-Za-z0-9_]+):", text, re.M) if substr in s]
    out = []
    for sym in syms:
        body = kernel_body(text, sym)
        ins = [ln.strip() for ln in body.splitlines() if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
        cnt = {"total": len(ins)}
        for k, pre in (("valu", "v_"), ("salu", "s_"), ("vmem", ("global_", "buffer_", "flat_")), ("lds", "ds_")):
            cnt[k] = sum(1 for x in ins if x.startswith(pre))
        tail = text[text.index("\n" + sym + ":"):]
        vg = re.search(r"; NumVgprs: (\d+)", tail)
        sg = re.search(r"; NumSgprs: (\d+)", tail)
        cnt["vgprs"] = int(vg.group(1)) if vg else None
        cnt["sgprs"] = int(sg.group(1)) if sg else None
        out.append((sym, cnt))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--kernel", default="k_stepILb1ELi1ELb0ELi5E")
    a = ap.parse_args()
    for f in a.files:
        for sym, c in stats(f, a.kernel):
            print(f, sym[:48], " ".join(f"{k}={v}" for k, v in c.items()))
