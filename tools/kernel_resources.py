#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / spill / LDS / occupancy table of a HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage, device-only compile, no GPU needed).

usage: tools/kernel_resources.py pyratslam_amd/csrc/posecell.hip [name-filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
extra = {'posecell.hip': ['-fno-slp-vectorize'],
         'view_templates.hip': ['-mllvm', '-amdgpu-atomic-optimizer-strategy=None']}
cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-x', 'hip',
       f'-I{ROOT}/include', f'-I{ROOT}/pyratslam_amd/csrc', '--cuda-device-only', '-c', src,
       '-o', '/dev/null', '-Rpass-analysis=kernel-resource-usage', *extra.get(os.path.basename(src), [])]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r'remark: (.*?) \[-Rpass', line)
    if not m:
        continue
    msg = m.group(1).strip()
    if msg.startswith('Function Name:'):
        name = subprocess.run(['c++filt'], input=msg.split(':', 1)[1].strip(),
                              capture_output=True, text=True).stdout.strip()
        name = re.sub(r'\(anonymous namespace\)::', '', name).split('(')[0]
        cur = {'name': name}
        rows.append(cur)
    elif cur is not None and ':' in msg:
        k, v = msg.split(':', 1)
        cur[k.strip()] = v.strip()
keys = ['VGPRs', 'AGPRs', 'ScratchSize [bytes/lane]', 'TotalSGPRs', 'SGPRs Spill', 'VGPRs Spill', 'LDS Size [bytes/block]', 'Occupancy [waves/SIMD]']
print('| kernel | ' + ' | '.join(k.split(' [')[0] for k in keys) + ' |')
print('|---' * (len(keys) + 1) + '|')
for r in rows:
    if flt in r['name']:
        print('| %s | ' % r['name'] + ' | '.join(r.get(k, '') for k in keys) + ' |')
