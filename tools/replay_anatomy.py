#!/usr/bin/env python3
"""Where the config-5 replay's time goes (GPU box): the synthetic ROS stream through
RatslamReplay with each callback's pieces timed -- pose-cell run()/update, the frame's
host subsample, the library call (rs_vt_match_batch) and the Python bookkeeping."""
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pyratslam_amd import replay, synthetic  # noqa: E402
from pyratslam_amd.view_templates import ViewTemplates  # noqa: E402

acc = defaultdict(float)
cnt = defaultdict(int)


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t0
            cnt[name] += 1
    return w


def main():
    events = synthetic.ros_stream(600, seed=0)
    replay.RatslamReplay(device=0).replay_events(events[:40])
    for rnd in range(2):
        acc.clear()
        cnt.clear()
        r = replay.RatslamReplay(device=0)
        r.vts.subsample = timed('subsample', r.vts.subsample)
        r.vts.match_templates = timed('match_templates', r.vts.match_templates)
        r.vts._record = timed('vts_record', r.vts._record)
        r.vis_callback = timed('vis_callback', r.vis_callback)
        r.pcn.run = timed('pcn_run', r.pcn.run)
        r.em.update = timed('em_update', r.em.update)
        r.drain = timed('drain', r.drain)
        t0 = time.perf_counter()
        r.replay_events(events)
        total = time.perf_counter() - t0
        out = {'total_ms': round(1e3 * total, 2), 'messages_per_s': round(len(events) / total),
               'templates': len(r.vts.templates)}
        for k in acc:
            out[k] = {'calls': cnt[k], 'us_per_call': round(1e6 * acc[k] / cnt[k], 2),
                      'ms': round(1e3 * acc[k], 2)}
        print(json.dumps(out))


if __name__ == '__main__':
    main()
