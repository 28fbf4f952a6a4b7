"""Check the chain kernels' inline-asm weight reads (sa_chain.hip ASMR): between an asm
ds_read_b128 and the s_waitcnt that covers it, no other instruction may read or write its
destination registers (a copy or use there would see the old bytes), and no branch may carry a
pending read to a target that does not wait for it first.

Run by the build (csrc/Makefile: the device assembly of sa_chain.hip, every PN2_CHAIN_SIGS
instance; a violation fails the build) and by hand:
    python tools/check_asm_reads.py <kernel .s>
Exit status 1 on any violation."""
import re
import sys


def _regs(line):
    regs = set()
    for a, b in re.findall(r'v\[(\d+):(\d+)\]', line):
        regs.update(range(int(a), int(b) + 1))
    for a in re.findall(r'\bv(\d+)\b', line):
        regs.add(int(a))
    return regs


def _covered(pending, n):
    """After s_waitcnt lgkmcnt(n) the n youngest LDS ops may still be in flight (they complete
    in order): are all asm reads among the older ones?"""
    young = pending[len(pending) - n:] if n else []
    return not any(dst for _, dst in young)


def check(src, out=sys.stdout):
    bad = 0
    for m in re.finditer(r'^(_ZN3pn215sa_chain_kernel\S+):\s*$', src, re.M):
        st = m.end()
        en = src.index('.Lfunc_end', st)
        body = [ln.strip() for ln in src[st:en].splitlines()]
        labels = {ln[:-1]: i for i, ln in enumerate(body) if ln.endswith(':') and not ln.startswith(';')}

        def target_waits(label, pending):
            # the first instruction at the branch target must be a wait covering the reads
            i = labels.get(label)
            if i is None:
                return False
            for ln in body[i + 1:]:
                if not ln or ln.startswith(';') or ln.startswith('.') or ln.endswith(':'):
                    continue
                mm = re.match(r's_waitcnt\b.*lgkmcnt\((\d+)\)', ln)
                return bool(mm) and _covered(pending, int(mm.group(1)))
            return False

        pending = []  # (line, destination regs of an asm read, or an empty set) oldest first
        in_asm = False
        name = m.group(1)[:70]
        for i, ln in enumerate(body):
            if ln.startswith(';;#ASMSTART'):
                in_asm = True
                continue
            if ln.startswith(';;#ASMEND'):
                in_asm = False
                continue
            if not ln or ln.startswith(';') or ln.startswith('.') or ln.endswith(':'):
                continue
            op = ln.split()[0]
            if op == 's_waitcnt' and 'lgkmcnt' in ln:
                n = int(re.search(r'lgkmcnt\((\d+)\)', ln).group(1))
                pending = pending[len(pending) - n:] if n else []
                continue
            live = any(dst for _, dst in pending)
            if live and (op.startswith('s_cbranch') or op == 's_branch' or op == 's_setpc_b64'):
                tgt = ln.split()[-1] if op != 's_setpc_b64' else None
                if tgt is None or not target_waits(tgt, pending):
                    print(name, 'line', i, 'branches with a pending asm read to', tgt, ':', ln, file=out)
                    bad += 1
            if live and op == 's_endpgm':
                print(name, 'line', i, 'ends with a pending asm read', file=out)
                bad += 1
            regs = _regs(ln)
            for (j, dst) in pending:
                if regs & dst:
                    print(name, 'line', i, 'touches pending read from line', j, ':', ln, file=out)
                    bad += 1
                    break
            if in_asm and op == 'ds_read_b128':
                a, b = re.search(r'v\[(\d+):(\d+)\]', ln).groups()
                pending.append((i, set(range(int(a), int(b) + 1))))
            elif op.startswith('ds_'):
                pending.append((i, set()))
    return bad


if __name__ == "__main__":
    n = check(open(sys.argv[1]).read())
    print('violations:', n)
    sys.exit(1 if n else 0)
