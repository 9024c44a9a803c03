"""Static check of a kernel's scratch (spill) traffic in compiler assembly (hipcc -S): the
round-1 four-wave fused-kernel fault.

For one kernel: every scratch access's bounds against the private segment, flat (generic)
accesses, and a reaching-definitions pass over the control-flow graph per scratch dword --
for every reload, the stores that can reach each of its dwords.  A reload whose dword can be
reached by the entry (no store on some path) or by a store of another slot layout (base
offset / width) than its own would read a value that is not the one spilled.

    python tools/scratch_check.py <file.s> <kernel symbol> <private segment bytes>
"""
import collections
import re
import sys


def parse(path, sym):
    lines, on = [], False
    for ln in open(path):
        if ln.startswith(sym + ":"):
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end"):
                break
            lines.append(ln.rstrip("\n"))
    return lines


def blocks(lines):
    """Basic blocks: (label, [instructions]); a label or a control-flow instruction ends one."""
    out, cur, lab = [], [], "__entry"
    for ln in lines:
        s = ln.split(";")[0].strip()
        m = re.match(r"^(\.L[\w$.]+):", s)
        if m:
            out.append((lab, cur))
            lab, cur = m.group(1), []
            continue
        if not s or s.startswith("."):
            continue
        cur.append(s)
        op = s.split()[0]
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op in ("s_setpc_b64", "s_endpgm"):
            out.append((lab, cur))
            lab, cur = f"__ft{len(out)}", []
    out.append((lab, cur))
    return [(l, b) for l, b in out if b or l.startswith(".L")]


def successors(bl):
    idx = {l: i for i, (l, _) in enumerate(bl)}
    succ = []
    for i, (l, ins) in enumerate(bl):
        nxt = [i + 1] if i + 1 < len(bl) else []
        if not ins:
            succ.append(nxt)
            continue
        last = ins[-1]
        op = last.split()[0]
        if op == "s_endpgm":
            succ.append([])
        elif op == "s_branch":
            succ.append([idx[last.split()[1]]])
        elif op.startswith("s_cbranch"):
            succ.append([idx[last.split()[1]]] + nxt)
        elif op == "s_setpc_b64":
            tgt = None
            for s in reversed(ins):
                m = re.search(r"\((\.L[\w$.]+)-\.L", s)
                if m:
                    tgt = m.group(1)
                    break
            succ.append([idx[tgt]] if tgt in idx else [])
        else:
            succ.append(nxt)
    return succ


ACC = re.compile(r"^scratch_(load|store)_dword(x(\d))?\s+(\S+),\s*(\S+),\s*(\S+)(?:\s+offset:(\d+))?")


def main():
    path, sym, seg = sys.argv[1], sys.argv[2], int(sys.argv[3])
    lines = parse(path, sym)
    bl = blocks(lines)
    succ = successors(bl)
    flat = sum(1 for _, ins in bl for s in ins if s.startswith("flat_"))
    accs = []          # (block, position, kind, offset, width, dynamic address)
    for b, (_, ins) in enumerate(bl):
        for p, s in enumerate(ins):
            m = ACC.match(s)
            if m:
                kind, n = m.group(1), int(m.group(3) or 1)
                vaddr = m.group(4) if kind == "load" else m.group(4)
                saddr = m.group(6)
                dyn = not (vaddr == "off" and saddr == "off") if kind == "store" else not (m.group(5) == "off" and saddr == "off")
                accs.append((b, p, kind, int(m.group(7) or 0), n, dyn))
    dyn = sum(1 for a in accs if a[5])
    over = [a for a in accs if a[3] + 4 * a[4] > seg]
    # reaching definitions per dword: ids of stores (-1 = the kernel's entry, nothing stored)
    store_id = {}
    for a in accs:
        if a[2] == "store":
            store_id[(a[0], a[1])] = len(store_id)
    meta = {store_id[(a[0], a[1])]: (a[3], a[4]) for a in accs if a[2] == "store"}
    dwords = sorted({a[3] + 4 * k for a in accs for k in range(a[4])})
    by_block = collections.defaultdict(list)
    for a in accs:
        by_block[a[0]].append(a)
    IN = [None] * len(bl)
    IN[0] = {d: frozenset([-1]) for d in dwords}

    def transfer(b, state):
        st = dict(state)
        for a in sorted(by_block[b], key=lambda x: x[1]):
            if a[2] == "store":
                for k in range(a[4]):
                    st[a[3] + 4 * k] = frozenset([store_id[(a[0], a[1])]])
        return st

    work = [0]
    OUT = [None] * len(bl)
    while work:
        b = work.pop()
        o = transfer(b, IN[b])
        if o == OUT[b]:
            continue
        OUT[b] = o
        for s in succ[b]:
            if IN[s] is None:
                IN[s] = dict(o)
                work.append(s)
            else:
                merged = {d: IN[s][d] | o[d] for d in dwords}
                if merged != IN[s]:
                    IN[s] = merged
                    work.append(s)
    bad_entry, bad_mix = [], []
    for b in range(len(bl)):
        if IN[b] is None:
            continue
        st = dict(IN[b])
        for a in sorted(by_block[b], key=lambda x: x[1]):
            if a[2] == "store":
                for k in range(a[4]):
                    st[a[3] + 4 * k] = frozenset([store_id[(a[0], a[1])]])
                continue
            for k in range(a[4]):
                rs = st[a[3] + 4 * k]
                if -1 in rs:
                    bad_entry.append((bl[b][0], bl[b][1][a[1]]))
                if any(meta[i] != (a[3], a[4]) for i in rs if i >= 0):
                    bad_mix.append((bl[b][0], bl[b][1][a[1]], sorted({meta[i] for i in rs if i >= 0})))
    unreached = sum(1 for x in IN if x is None)
    print(f"{sym}: {len(bl)} blocks ({unreached} unreachable), {len(accs)} scratch accesses "
          f"({sum(1 for a in accs if a[2] == 'load')} loads), {dyn} with a register address, {flat} flat accesses")
    print(f"private segment {seg} B; largest access end {max(a[3] + 4 * a[4] for a in accs)} B; "
          f"accesses past the segment: {len(over)}")
    print(f"reloads reachable from the entry without a store: {len(bad_entry)}")
    for x in bad_entry[:10]:
        print("   ", x)
    print(f"reloads of a dword reachable from a store of another slot layout: {len(bad_mix)}")
    for x in bad_mix[:10]:
        print("   ", x)


if __name__ == "__main__":
    main()
