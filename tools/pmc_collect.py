#!/usr/bin/env python3
"""Summarise tools/profile_r2.sh output into profiles/ (run where gpurun_out/ is).

Per configuration: kernel durations from the kernel trace (rocprofv3 --stats),
HBM bytes per dispatch from the FETCH_SIZE and WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md section HBM prescribes (FETCH_SIZE reports half of the bytes
of a wide coalesced read on gfx950, so it is doubled; both counters are KiB;
Infinity-Cache hits are counted too, so this is an upper bound on DRAM bytes):
  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024,
and the SQ pass (SQ_INSTS_VALU wave-instructions; the wave-cycle split
SQ_WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY).

Writes profiles/<tag>_pmc_summary.json, profiles/<tag>_kernel_summary.md and
profiles/pmc_traffic.json (what bench.py reads for its roofline fields).

usage: tools/pmc_collect.py --dir gpurun_out/prof_<tag> --tag r2_v1 [--out profiles]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import shutil

SCANS = {'headline': (1000, 10240), 'stress': (10000, 5120), 'library': (100000, 2048)}
PCS = {'pc64': ('halo', [64, 64, 36]), 'pc128': ('cols', [128, 128, 72])}


def short(name):
    name = re.sub(r'\(anonymous namespace\)::', '', name)
    name = re.sub(r'^void ', '', name)
    return name.split('(')[0]


def find(d, pattern):
    hits = glob.glob(os.path.join(d, '**', pattern), recursive=True)
    return hits[0] if hits else None


def trace_stats(d):
    """Per kernel: rocprofv3's --stats summary, plus the median over the per-dispatch
    kernel trace (the first dispatches of a process run while the clocks ramp up, which
    pulls the average above the steady state the bench's timed steps see)."""
    f = find(d, '*kernel_stats.csv')
    out = {}
    if not f:
        return out
    for r in csv.DictReader(open(f)):
        out[short(r['Name'])] = {'calls': int(r['Calls']), 'avg_us': float(r['AverageNs']) / 1e3,
                                 'min_us': float(r['MinNs']) / 1e3, 'max_us': float(r['MaxNs']) / 1e3,
                                 'pct': float(r['Percentage'])}
    t = find(d, '*kernel_trace.csv')
    if t:
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(t)):
            per[short(r['Kernel_Name'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
        for k, v in per.items():
            if k in out:
                v.sort()
                out[k]['median_us'] = v[len(v) // 2]
    return out


def counters(d):
    f = find(d, '*counter_collection.csv')
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    if not f:
        return per
    for r in csv.DictReader(open(f)):
        per[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    return per


def summarise(base, c):
    stats = trace_stats(os.path.join(base, c + '_trace'))
    fetch = counters(os.path.join(base, c + '_fetch'))
    write = counters(os.path.join(base, c + '_write'))
    sq = counters(os.path.join(base, c + '_sq'))
    kernels = {}
    for k in sorted(set(stats) | set(fetch) | set(write) | set(sq)):
        e = {'trace': stats.get(k)}
        f = fetch.get(k, {}).get('FETCH_SIZE', [])
        w = write.get(k, {}).get('WRITE_SIZE', [])
        if f and w:
            fk, wk = sum(f) / len(f), sum(w) / len(w)
            e.update({'fetch_kib_raw': fk, 'write_kib': wk, 'dispatches': len(f),
                      'hbm_bytes_per_dispatch': (2 * fk + wk) * 1024})
        s = {n: sum(v) / len(v) for n, v in sq.get(k, {}).items() if v}
        if s:
            e['sq'] = s
            wc = s.get('SQ_WAVE_CYCLES', 0)
            if wc > 0:
                e['wave_cycle_split'] = {n: s.get(ctr, 0) / wc for n, ctr in (
                    ('issuing', 'SQ_ACTIVE_INST_ANY'), ('issue_stall', 'SQ_WAIT_INST_ANY'),
                    ('waitcnt_or_barrier', 'SQ_WAIT_ANY'))}
        kernels[k] = e
    return kernels


def traffic_of(configs, tag):
    """pmc_traffic.json (what bench.py reads) from the per-configuration kernels.
    A scan configuration's profiled kernel is its 64x32-template instantiation
    (vt_scan_plane_kernel<64, ...>): the 32x32 scans that warm the clocks first
    run more, shorter dispatches and are not the configuration's kernel."""
    traffic = {'source': f'{tag}_pmc_summary.json', 'scans': {}, 'pose_cell': {}}
    for c, ks in configs.items():
        if c in SCANS:
            scan = [k for k in ks if k.startswith('vt_scan') and '<64' in k and ks[k].get('trace')]
            if not scan:
                continue
            k = max(scan, key=lambda n: ks[n]['trace']['calls'])
            e = ks[k]
            traffic['scans'][c] = {
                'kernel': k, 'templates_per_launch': SCANS[c][0], 'queries': SCANS[c][1],
                'kernel_us_rocprof': e['trace'].get('median_us', e['trace']['avg_us']),
                'kernel_us_rocprof_avg': e['trace']['avg_us'],
                'valu_insts_per_launch': e.get('sq', {}).get('SQ_INSTS_VALU'),
                'hbm_bytes_per_launch': e.get('hbm_bytes_per_dispatch'),
                'wave_cycle_split': e.get('wave_cycle_split'),
                'source': f'{tag}_pmc_summary.json'}
        elif c in PCS and PCS[c][0] == 'halo':
            # one launch per step; the finishing kernel once per run() call, its time and
            # bytes spread over the call's steps
            form, shape = PCS[c]
            st = [k for k in ks if k.startswith('pc_step_halo') and ks[k].get('trace')]
            if not st:
                continue
            st = max(st, key=lambda n: ks[n]['trace']['calls'])
            fi = [k for k in ks if k.startswith('pc_halo_finish') and ks[k].get('trace')]
            hb = ks[st].get('hbm_bytes_per_dispatch')
            rec = {'shape': shape, 'kernels': [st] + fi[:1],
                   'kernel_us_rocprof': {'step': ks[st]['trace'].get('median_us', ks[st]['trace']['avg_us'])},
                   'hbm_bytes_per_step': hb, 'source': f'{tag}_pmc_summary.json'}
            if fi and hb:
                f = ks[fi[0]]
                per = f['trace']['calls'] / ks[st]['trace']['calls']
                rec['kernel_us_rocprof']['finish_per_step'] = per * f['trace'].get('median_us', f['trace']['avg_us'])
                if f.get('hbm_bytes_per_dispatch'):
                    rec['hbm_bytes_per_step'] = hb + per * f['hbm_bytes_per_dispatch']
            traffic['pose_cell'][form] = rec
        elif c in PCS:
            form, shape = PCS[c]
            ex = [k for k in ks if k.startswith('pc_excite') and ks[k].get('trace')]
            pa = [k for k in ks if k.startswith('pc_path') and ks[k].get('trace')]
            if not (ex and pa):
                continue
            ex = max(ex, key=lambda n: ks[n]['trace']['calls'])
            pa = max(pa, key=lambda n: ks[n]['trace']['calls'])
            hb = [ks[n].get('hbm_bytes_per_dispatch') for n in (ex, pa)]
            traffic['pose_cell'][form] = {
                'shape': shape, 'kernels': [ex, pa],
                'kernel_us_rocprof': {'excite': ks[ex]['trace'].get('median_us', ks[ex]['trace']['avg_us']),
                                      'path': ks[pa]['trace'].get('median_us', ks[pa]['trace']['avg_us'])},
                'hbm_bytes_per_step': sum(hb) if all(hb) else None,
                'hbm_bytes_per_kernel': {'excite': hb[0], 'path': hb[1]} if all(hb) else None,
                'source': f'{tag}_pmc_summary.json'}
    return traffic


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dir', default='')
    ap.add_argument('--resummarise', action='store_true',
                    help='rewrite pmc_traffic.json from profiles/<tag>_pmc_summary.json')
    ap.add_argument('--tag', required=True)
    ap.add_argument('--out', default='profiles')
    a = ap.parse_args()
    summary = {'tag': a.tag, 'method': __doc__.strip().splitlines()[2:11], 'configs': {}}
    if a.resummarise:  # rebuild pmc_traffic.json from an existing summary (no raw data)
        summary = json.load(open(os.path.join(a.out, f'{a.tag}_pmc_summary.json')))
        with open(os.path.join(a.out, 'pmc_traffic.json'), 'w') as fh:
            json.dump(traffic_of(summary['configs'], a.tag), fh, indent=1)
        return
    for c in list(SCANS) + list(PCS):
        if not glob.glob(os.path.join(a.dir, c + '_*')):
            continue
        summary['configs'][c] = summarise(a.dir, c)
    traffic = traffic_of(summary['configs'], a.tag)
    # the raw inputs of every figure, tracked: each configuration's rocprofv3
    # kernel_stats.csv and its per-kernel counter averages (one row per kernel and
    # counter) under profiles/<tag>/, named in pmc_traffic.json's source fields
    raw = os.path.join(a.out, a.tag)
    os.makedirs(raw, exist_ok=True)
    for c in summary['configs']:
        f = find(os.path.join(a.dir, c + '_trace'), '*kernel_stats.csv')
        if f:
            shutil.copy(f, os.path.join(raw, f'{c}_kernel_stats.csv'))
        t = find(os.path.join(a.dir, c + '_trace'), '*kernel_trace.csv')
        if t:  # per dispatch: name, start, end (the medians' input)
            with open(t) as src, open(os.path.join(raw, f'{c}_kernel_trace.csv'), 'w', newline='') as dst:
                wr = csv.writer(dst)
                wr.writerow(['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
                for r in csv.DictReader(src):
                    wr.writerow([short(r['Kernel_Name']), r['Start_Timestamp'], r['End_Timestamp']])
        with open(os.path.join(raw, f'{c}_counters.csv'), 'w', newline='') as fh:
            wr = csv.writer(fh)
            wr.writerow(['pass', 'kernel', 'counter', 'dispatches', 'mean_value'])
            for ps in ('fetch', 'write', 'sq'):
                for k, cs in sorted(counters(os.path.join(a.dir, f'{c}_{ps}')).items()):
                    for n, v in sorted(cs.items()):
                        wr.writerow([ps, k, n, len(v), repr(sum(v) / len(v))])
    f = find(os.path.join(a.dir, 'bench_trace'), '*kernel_stats.csv')
    if f:
        shutil.copy(f, os.path.join(raw, 'bench_kernel_stats.csv'))
    for c, rec in list(traffic['scans'].items()) + list(traffic['pose_cell'].items()):
        cfg = c if c in SCANS else {'rows': 'pc64', 'halo': 'pc64', 'cols': 'pc128'}[c]
        rec['kernel_us_source'] = (f'profiles/{a.tag}/{cfg}_kernel_trace.csv (median over the dispatches; '
                                   f'the --stats average is kernel_us_rocprof_avg, {cfg}_kernel_stats.csv)')
        rec['counter_source'] = f'profiles/{a.tag}/{cfg}_counters.csv'
    bench = trace_stats(os.path.join(a.dir, 'bench_trace'))
    if bench:
        summary['bench_command'] = {'command': 'python bench.py', 'kernels': bench}
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, f'{a.tag}_pmc_summary.json'), 'w') as fh:
        json.dump(summary, fh, indent=1)
    with open(os.path.join(a.out, 'pmc_traffic.json'), 'w') as fh:
        json.dump(traffic, fh, indent=1)
    lines = [f'# rocprofv3 summary, {a.tag}', '',
             'Per configuration (tools/profile_r2.sh, tools/scan_profile.py): kernel trace + '
             'stats and PMC passes; HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch.', '']
    for c, ks in summary['configs'].items():
        lines += [f'## {c}', '', '| kernel | calls | avg us | min us | max us | HBM bytes/dispatch | '
                  'VALU insts/dispatch | issuing / stall / wait |', '|---|---|---|---|---|---|---|---|']
        for k, e in sorted(ks.items(), key=lambda kv: -((kv[1]['trace'] or {}).get('pct', 0))):
            t = e['trace'] or {}
            hb = e.get('hbm_bytes_per_dispatch')
            vi = e.get('sq', {}).get('SQ_INSTS_VALU')
            ws = e.get('wave_cycle_split')
            lines.append('| %s | %s | %.2f | %.2f | %.2f | %s | %s | %s |' % (
                k, t.get('calls', '-'), t.get('avg_us', 0), t.get('min_us', 0), t.get('max_us', 0),
                '%.3e' % hb if hb else '-', '%.4g' % vi if vi else '-',
                '%.2f / %.2f / %.2f' % (ws['issuing'], ws['issue_stall'], ws['waitcnt_or_barrier'])
                if ws else '-'))
        lines.append('')
    if bench:
        lines += ['## bench command (`python bench.py`, kernel trace + stats)', '',
                  '| kernel | calls | avg us | min us | max us | % time |', '|---|---|---|---|---|---|']
        for k, t in sorted(bench.items(), key=lambda kv: -kv[1]['pct']):
            lines.append('| %s | %d | %.2f | %.2f | %.2f | %.1f |' % (
                k, t['calls'], t['avg_us'], t['min_us'], t['max_us'], t['pct']))
    with open(os.path.join(a.out, f'{a.tag}_kernel_summary.md'), 'w') as fh:
        fh.write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


if __name__ == '__main__':
    main()
