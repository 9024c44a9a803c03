"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (the packet walks'
loops: SALU / VALU / SMEM / VMEM / branch counts per block, with the loop depth the compiler
annotates), for comparing code shapes of a kernel between builds on the CPU.

    python tools/isa_blocks.py listing.s <kernel-name-regex>"""
import argparse
import re


def kernel_body(path, pat):
    lines = open(path).read().split("\n")
    rx = re.compile(pat)
    for i, l in enumerate(lines):
        if not l or l[0].isspace() or l.startswith(".") or ":" not in l:
            continue
        name, rest = l.split(":", 1)
        if rx.search(name) and rest.strip().startswith(";"):
            j = i
            while not lines[j].startswith(".Lfunc_end"):
                j += 1
            return name, lines[i:j]
    raise SystemExit("kernel not found")


def classify(ins):
    op = ins.split()[0]
    if op.startswith(("s_cbranch", "s_branch", "s_setpc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_endpgm")):
        return "other"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("listing")
    ap.add_argument("kernel")
    a = ap.parse_args()
    name, body = kernel_body(a.listing, a.kernel)
    print(name)
    blocks, cur = [], None
    for l in body[1:]:
        s = l.strip()
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?(.*)$", s)
        if m:
            cur = {"name": m.group(1).lstrip("; "), "note": m.group(2).strip(), "n": {}}
            blocks.append(cur)
            continue
        if not s or s.startswith((";", ".")) or cur is None:
            if cur is not None and "Loop" in s:
                cur["note"] += " " + s
            continue
        c = classify(s)
        cur["n"][c] = cur["n"].get(c, 0) + 1
        if s.startswith("scratch_"):
            cur["n"]["scratch"] = cur["n"].get("scratch", 0) + 1
    tot = {}
    for b in blocks:
        n = b["n"]
        for k, v in n.items():
            tot[k] = tot.get(k, 0) + v
        depth = re.findall(r"Depth=(\d)", b["note"])
        print(f"{b['name']:12s} d{max(depth) if depth else 0} " +
              " ".join(f"{k}={n.get(k, 0)}" for k in ("salu", "valu", "smem", "vmem", "lds", "branch")) +
              (f" scratch={n['scratch']}" if n.get("scratch") else ""))
    print("total", tot)


if __name__ == "__main__":
    main()
