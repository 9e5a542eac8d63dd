#!/usr/bin/env python3
"""Static check of hand-counted vector-memory loads in a gfx9 device assembly
listing (hipcc -S --cuda-device-only): for every kernel, walk its instructions
in text order, keep the destination VGPRs of the vector-memory loads still in
flight (vmcnt counts them, and the stores and returnless atomics issued between
them, in issue order) and report any instruction that reads
or writes such a register before an `s_waitcnt vmcnt(N)` has retired the load.

A hit is a real hazard on straight-line code: a read sees the register before
the data lands, a write is clobbered when the data lands.  (The walk ignores
conditional branches, so a hit across a loop back edge is approximate; after an
unconditional jump only inline-asm loads stay tracked.)

This is the evidence behind DESIGN.md's account of the round-1 illegal-address
fault: the inline-asm window loads of the old stream kernels (commit f7be589^)
told hipcc that their destination was written at the asm statement, so the
register allocator was free to read, copy or reuse it while the load was still
in flight.

usage: python tools/asm_load_hazards.py LISTING.s [--kernel SUBSTR] [--asm-only]
"""
import argparse
import re
import sys

LOAD = re.compile(r'^(global_load|buffer_load|flat_load|scratch_load)\w*\s+(\S+?),')
WAIT = re.compile(r'^s_waitcnt\b(.*)')
# vector-memory operations without a VGPR destination that still take a vmcnt slot
VMEM_NODEST = re.compile(r'^(global_store|buffer_store|flat_store|scratch_store)\w*\s|'
                         r'^(global_atomic|buffer_atomic|flat_atomic)\w*\s(?!.*\b(sc0|glc)\b)')
REG = re.compile(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b')


def regs(text):
    out = set()
    for a, b, c in REG.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def kernels(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r'^(_Z\S+):', ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(ln)
            if ln.strip().startswith('.Lfunc_end'):
                yield cur, body
                cur, body = None, []


def scan(name, body, asm_only):
    inflight = []            # [(dest regs, line no, from_asm)] in issue order
    in_asm = False
    hits = []
    for no, raw in enumerate(body):
        s = raw.split(';')[0].strip()
        if ';;#ASMSTART' in raw:
            in_asm = True
            continue
        if ';;#ASMEND' in raw:
            in_asm = False
            continue
        if not s or s.startswith('.') or s.endswith(':'):
            continue
        if re.match(r'^(s_branch|s_setpc_b64|s_endpgm)\b', s):
            # the text after an unconditional jump is not its fall-through: the
            # compiler's own loads are waited for on the real path (hipcc places
            # their waits on the CFG); keep tracking only the asm loads it cannot see
            inflight = [x for x in inflight if x[2]]
            continue
        w = WAIT.match(s)
        if w:
            m = re.search(r'vmcnt\((\d+)\)', w.group(1))
            if m:
                keep = int(m.group(1))
                while len(inflight) > keep:
                    inflight.pop(0)
            continue
        m = LOAD.match(s)
        ops = s.split(None, 1)[1] if ' ' in s else ''
        if m and ('_lds' in s.split()[0] or re.search(r'\blds\b', ops)):
            # LDS-DMA (global_load_lds_*, buffer_load ... lds): no VGPR destination, the
            # operands are addresses read at issue; it still holds a vmcnt slot
            dest, srcs = set(), regs(ops)
        elif m:
            dest = regs(m.group(2))
            srcs = regs(ops[len(m.group(2)):])
        else:
            parts = ops.split(',', 1)
            dest = regs(parts[0]) if parts and parts[0] else set()
            srcs = regs(parts[1]) if len(parts) > 1 else set()
            if s.startswith(('global_store', 'buffer_store', 'ds_write', 'ds_store', 'flat_store',
                             'scratch_store')):
                srcs, dest = regs(ops), set()
        for d, lno, from_asm in inflight:
            if asm_only and not from_asm:
                continue
            if d & srcs:
                hits.append((no, 'read', sorted(d & srcs), lno, s))
            if d & dest and not m:  # a later load lands after it (in-order return)
                hits.append((no, 'write', sorted(d & dest), lno, s))
        if m:
            inflight.append((dest, no, in_asm))
        elif VMEM_NODEST.match(s):
            # on gfx9 stores and returnless atomics count in vmcnt too: they hold a slot
            # (no destination), so `vmcnt(N)` after them retires loads issued earlier
            inflight.append((set(), no, in_asm))
    return hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('listing')
    ap.add_argument('--kernel', default='')
    ap.add_argument('--asm-only', action='store_true', help='only loads issued by inline asm')
    ap.add_argument('--show', type=int, default=3)
    a = ap.parse_args()
    lines = open(a.listing).read().splitlines()
    total = 0
    for name, body in kernels(lines):
        if a.kernel not in name:
            continue
        hits = scan(name, body, a.asm_only)
        total += len(hits)
        print(f'{len(hits):5d}  {name[:110]}')
        for no, kind, r, lno, s in hits[:a.show]:
            print(f'         +{no}: {kind} of v{r} (load at +{lno} in flight): {s}')
    print('total hazards:', total)
    return 0


if __name__ == '__main__':
    sys.exit(main())
