"""bench.py's roofline inputs (profiles/pmc_traffic.json) describe the kernels the
bench launches, and the fractions they give are physical (CPU only)."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _traffic():
    return json.load(open(os.path.join(ROOT, 'profiles', 'pmc_traffic.json')))


def test_scan_records_name_the_64x32_instantiation():
    tj = _traffic()
    for key in ('headline', 'stress', 'library'):
        rec = tj['scans'][key]
        assert rec['kernel'].startswith('vt_scan_plane_kernel<64'), (key, rec['kernel'])
        # the method's own VALU count: 8 bitop3 + 1 bcnt per 32 byte
        # pairs, 192 unit pairs per column group and compare, 4 column groups, per
        # 64 templates of a wave -- the PMC count sits within 20% above it
        core = 9 * 192 * 4 * rec['templates_per_launch'] * rec['queries'] / 64
        assert core <= rec['valu_insts_per_launch'] <= 1.2 * core, (key, core, rec['valu_insts_per_launch'])


def test_scan_roofline_fraction_is_physical():
    tj = _traffic()
    rec = tj['scans']['headline']
    tv = {'templates_per_launch': rec['templates_per_launch'], 'queries_per_launch': rec['queries'],
          'kernel': 'vt_scan_plane_kernel', 'scan_ms': rec['kernel_us_rocprof'] * 1e-3,
          'compares_per_launch': rec['templates_per_launch'] * rec['queries']}
    roof = bench.scan_roofline(tv, tj, 'headline')
    assert roof['bound'] == 'valu'
    assert 0.3 < roof['frac'] <= 1.0, roof['frac']
    # a record of another instantiation is not used
    other = json.loads(json.dumps(tj))
    other['scans']['headline']['kernel'] = 'vt_scan_plane_kernel<32, false>'
    assert bench.scan_roofline(tv, other, 'headline')['frac'] is None
