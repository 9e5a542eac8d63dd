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


def test_pose_cell_records_name_the_default_step_kernels():
    """The 64x64x36 record is the halo form's one step kernel (the bench's default form
    there), with PMC bytes per step of the order of the 24 B/cell the survey prices and a
    kernel time that fits the measured wall per step; the 128x128x72 record is the column
    form's excite + path pair."""
    tj = _traffic()
    halo = tj['pose_cell']['halo']
    assert halo['shape'] == [64, 64, 36]
    assert halo['kernels'][0].startswith(('pc_step_halo<false>', 'pc_step_halo<false, 36>'))   # (36: round 6's template)
    cells = 64 * 64 * 36
    assert 0.25 * 24 * cells < halo['hbm_bytes_per_step'] < 4 * 24 * cells
    assert 5.0 < halo['kernel_us_rocprof']['step'] < 20.0
    cols = tj['pose_cell']['cols']
    assert cols['shape'] == [128, 128, 72]
    assert [k.split('<')[0] for k in cols['kernels']] == ['pc_excite_cols', 'pc_path_cols']


def test_pmc_collect_halo_record():
    """tools/pmc_collect.py turns a profiled halo run (step kernel per step, the finishing
    kernel once per call) into per-step time and bytes."""
    import importlib.util
    spec = importlib.util.spec_from_file_location('pmc_collect', os.path.join(ROOT, 'tools', 'pmc_collect.py'))
    pc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pc)
    ks = {'pc_step_halo<false>': {'trace': {'calls': 400, 'avg_us': 9.2, 'median_us': 9.0},
                                  'hbm_bytes_per_dispatch': 2.0e6},
          'pc_halo_finish': {'trace': {'calls': 4, 'avg_us': 4.0, 'median_us': 4.0},
                             'hbm_bytes_per_dispatch': 1.0e6}}
    rec = pc.traffic_of({'pc64': ks}, 'tag')['pose_cell']['halo']
    assert rec['kernel_us_rocprof'] == {'step': 9.0, 'finish_per_step': 0.04}
    assert abs(rec['hbm_bytes_per_step'] - (2.0e6 + 0.01 * 1.0e6)) < 1e-6
