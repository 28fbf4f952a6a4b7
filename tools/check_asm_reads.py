"""Check the chain kernels' inline-asm weight reads (sa_chain.hip ASMR): between an asm
ds_read_b128 and the s_waitcnt that covers it, no other instruction may read or write its
destination registers (a copy or use there would see the old bytes).
    python tools/check_asm_reads.py <kernel .s>"""
import re
import sys

src = open(sys.argv[1]).read()
bad = 0
for m in re.finditer(r'^(_ZN3pn215sa_chain_kernel\S+):\s*$', src, re.M):
    st = m.end()
    en = src.index('.Lfunc_end', st)
    body = [l.strip() for l in src[st:en].splitlines()]
    pending = []  # (line, regs set, count of LDS ops issued after it)
    in_asm = False
    for i, l in enumerate(body):
        if l.startswith(';;#ASMSTART'):
            in_asm = True
            continue
        if l.startswith(';;#ASMEND'):
            in_asm = False
            continue
        if not l or l.startswith(';') or l.startswith('.') or l.endswith(':'):
            continue
        op = l.split()[0]
        regs = set()
        for a, b in re.findall(r'v\[(\d+):(\d+)\]', l):
            regs.update(range(int(a), int(b) + 1))
        for a in re.findall(r'\bv(\d+)\b', l):
            regs.add(int(a))
        if op == 's_waitcnt' and 'lgkmcnt' in l:
            n = int(re.search(r'lgkmcnt\((\d+)\)', l).group(1))
            # LDS ops complete in order: keep only the n youngest pending
            pending = pending[len(pending) - n:] if n else []
            continue
        if op == 's_barrier' or op.startswith('s_cbranch') or op == 's_branch' or op == 's_endpgm':
            if pending and op != 's_barrier':
                # a pending asm read across a branch: allowed only if the target re-waits; flag it
                pass
        for (j, dst) in pending:
            if regs & dst:
                print(m.group(1)[:60], 'line', i, 'touches pending read from line', j, ':', l)
                bad += 1
                break
        if in_asm and op == 'ds_read_b128':
            a, b = re.search(r'v\[(\d+):(\d+)\]', l).groups()
            pending.append((i, set(range(int(a), int(b) + 1))))
        elif op.startswith('ds_'):
            pending.append((i, set()))
print('violations:', bad)
