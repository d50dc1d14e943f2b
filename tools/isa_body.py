"""Instruction body of one kernel in a hipcc `--cuda-device-only -S` listing, labels renamed
to their order of appearance and the kernel's own name stripped, so two builds whose template
signatures differ (e.g. a removed template axis) can be compared instruction for instruction.

    python tools/isa_body.py listing.s <mangled-name-substring> [out.txt]

Prints the instruction count and VALU / SALU / LDS / branch counts; writes the body to out.txt.
"""
import re
import sys


def body(listing, key):
    s = open(listing).read()
    m = re.search(r"^(_Z\S*%s\S*):" % re.escape(key), s, re.M)
    if not m:
        raise SystemExit(f"no kernel matching {key}")
    name = m.group(1)
    i = m.end()
    j = s.index(".Lfunc_end", i)
    labels = {}
    out = []
    for line in s[i:j].split("\n"):
        t = line.split(";")[0].strip()
        if not t or t.startswith("."):
            if t.startswith(".LBB") and t.endswith(":"):
                labels.setdefault(t[:-1], f"L{len(labels)}")
                out.append(labels[t[:-1]] + ":")
            continue
        t = re.sub(r"\.LBB\w+", lambda x: labels.setdefault(x.group(0), f"L{len(labels)}"), t)
        out.append(t.replace(name, "K"))
    return name, out


def counts(lines):
    ins = [l for l in lines if not l.endswith(":")]
    op = [l.split()[0] for l in ins]
    return {"insts": len(ins), "valu": sum(o.startswith("v_") for o in op),
            "salu": sum(o.startswith("s_") and not o.startswith("s_cbranch") and o != "s_branch" for o in op),
            "lds": sum(o.startswith("ds_") for o in op),
            "branches": sum(o.startswith("s_cbranch") or o == "s_branch" for o in op)}


if __name__ == "__main__":
    name, b = body(sys.argv[1], sys.argv[2])
    print(name, counts(b))
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write("\n".join(b) + "\n")
