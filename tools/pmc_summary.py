#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/ (per-kernel time and HBM bytes).

HBM bytes per dispatch follow MI355X_MICROARCH.md section HBM: FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes (TCC slots), both in KiB;
FETCH_SIZE reports half of the bytes of a wide coalesced read on gfx950, so it
is doubled: hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Infinity-cache
hits are counted too, so this is an upper bound on DRAM bytes.

SQ counters (optional --sq DIR): SQ_INSTS_VALU per dispatch (wave-instructions),
the wave-cycle split (SQ_WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY,
quad-cycles) and GRBM_GUI_ACTIVE / 8 (cycles per XCD = the dispatch's clock span).

usage: tools/pmc_summary.py --fetch DIR --write DIR --trace DIR [--sq DIR] --round r1 [--out profiles]
"""
import argparse
import collections
import csv
import json
import os
import re


def short(name):
    name = re.sub(r'\(anonymous namespace\)::', '', name)
    name = re.sub(r'^void ', '', name)
    return name.split('(')[0]


def counters(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(path, 'run_counter_collection.csv'))):
        if r['Counter_Name'] == counter:
            per[short(r['Kernel_Name'])].append(float(r['Counter_Value']))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--fetch', required=True)
    ap.add_argument('--write', required=True)
    ap.add_argument('--trace', required=True)
    ap.add_argument('--sq', default=None)
    ap.add_argument('--round', default='r1')
    ap.add_argument('--out', default='profiles')
    ap.add_argument('--templates-per-gpu', type=int, default=1000)
    ap.add_argument('--queries', type=int, default=1024)
    a = ap.parse_args()
    fetch = counters(a.fetch, 'FETCH_SIZE')
    write = counters(a.write, 'WRITE_SIZE')
    sq_names = ('SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_WAVE_CYCLES', 'SQ_ACTIVE_INST_ANY',
                'SQ_WAIT_INST_ANY', 'SQ_WAIT_ANY', 'GRBM_GUI_ACTIVE')
    sq = {c: counters(a.sq, c) for c in sq_names} if a.sq else {}
    stats = {}
    for r in csv.DictReader(open(os.path.join(a.trace, 'run_kernel_stats.csv'))):
        stats[short(r['Name'])] = {'calls': int(r['Calls']), 'avg_us': float(r['AverageNs']) / 1e3,
                                   'min_us': float(r['MinNs']) / 1e3, 'max_us': float(r['MaxNs']) / 1e3,
                                   'pct': float(r['Percentage'])}
    kernels = {}
    for k in sorted(set(fetch) | set(write) | set(stats)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        e = {'trace': stats.get(k)}
        if f and w:
            fk = sum(f) / len(f)
            wk = sum(w) / len(w)
            e.update({'fetch_kib_raw': fk, 'write_kib': wk,
                      'hbm_bytes_per_dispatch': (2 * fk + wk) * 1024, 'dispatches': len(f)})
        sqk = {c: sum(v[k]) / len(v[k]) for c, v in sq.items() if v.get(k)}
        if sqk:
            e['sq'] = sqk
            if 'SQ_WAVE_CYCLES' in sqk and sqk['SQ_WAVE_CYCLES'] > 0:
                wc = sqk['SQ_WAVE_CYCLES']
                e['wave_cycle_split'] = {n: sqk.get(c, 0) / wc for n, c in (
                    ('issuing', 'SQ_ACTIVE_INST_ANY'), ('issue_stall', 'SQ_WAIT_INST_ANY'),
                    ('waitcnt_or_barrier', 'SQ_WAIT_ANY'))}
        kernels[k] = e
    os.makedirs(a.out, exist_ok=True)
    summary = {'round': a.round, 'method': __doc__.strip().splitlines()[2:7], 'kernels': kernels}
    with open(os.path.join(a.out, f'{a.round}_pmc_summary.json'), 'w') as fh:
        json.dump(summary, fh, indent=1)
    scan = [k for k in kernels if k.startswith('vt_scan') and 'hbm_bytes_per_dispatch' in kernels[k]]
    if scan:
        k = max(scan, key=lambda s: kernels[s]['dispatches'])
        # pose-cell steps: HBM bytes of one excite + one path dispatch (float32,
        # batched-run control), per step form -- rows (the 64x64x36 headline grid)
        # and stream (the 128x128x72 stress grid)
        pc = {}
        for form in ('rows', 'stream'):
            ex = [n for n in kernels if n.startswith(f'pc_excite_{form}<float')
                  and 'hbm_bytes_per_dispatch' in kernels[n]]
            pa = [n for n in kernels if n.startswith(f'pc_path_{form}<float') and 'PcCtlRing' in n
                  and 'hbm_bytes_per_dispatch' in kernels[n]]
            if ex and pa:
                ex = max(ex, key=lambda n: kernels[n]['dispatches'])
                pa = max(pa, key=lambda n: kernels[n]['dispatches'])
                pc[form] = {'kernels': [ex, pa], 'hbm_bytes_per_step':
                            kernels[ex]['hbm_bytes_per_dispatch'] + kernels[pa]['hbm_bytes_per_dispatch']}
        with open(os.path.join(a.out, 'pmc_traffic.json'), 'w') as fh:
            json.dump({'kernel': k, 'hbm_bytes_per_launch': kernels[k]['hbm_bytes_per_dispatch'],
                       'valu_insts_per_launch': kernels[k].get('sq', {}).get('SQ_INSTS_VALU'),
                       'templates_per_gpu': a.templates_per_gpu, 'queries': a.queries,
                       'pose_cell': pc, 'source': f'{a.round}_pmc_summary.json'}, fh, indent=1)
    lines = [f'# rocprofv3 summary, round {a.round}', '',
             '| kernel | calls | avg us | min us | max us | % time | HBM bytes/dispatch (2*FETCH+WRITE) |',
             '|---|---|---|---|---|---|---|']
    for k, e in sorted(kernels.items(), key=lambda kv: -(kv[1]['trace'] or {}).get('pct', 0)):
        t = e['trace'] or {}
        hb = e.get('hbm_bytes_per_dispatch')
        lines.append('| %s | %s | %.2f | %.2f | %.2f | %.1f | %s |' % (
            k, t.get('calls', '-'), t.get('avg_us', 0), t.get('min_us', 0), t.get('max_us', 0),
            t.get('pct', 0), '%.3e' % hb if hb else '-'))
    with open(os.path.join(a.out, f'{a.round}_kernel_summary.md'), 'w') as fh:
        fh.write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


if __name__ == '__main__':
    main()
