#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: VGPRs, scratch, occupancy per kernel."""
import re, subprocess, sys

def main(path):
    txt = open(path).read()
    rows, cur = [], None
    for line in txt.splitlines():
        m = re.search(r'Function Name: (\S+)', line)
        if m:
            cur = {'name': subprocess.run(['c++filt', m.group(1)], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
            continue
        for key, pat in (('vgpr', r'VGPRs: (\d+)'), ('scratch', r'ScratchSize \[bytes/lane\]: (\d+)'),
                         ('occ', r'Occupancy \[waves/SIMD\]: (\d+)')):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    for r in rows:
        name = re.sub(r'dpac::', '', r['name'])
        name = re.sub(r'\(.*', '', name)
        print(f"{r.get('vgpr', '?'):>4} vgpr  scratch {r.get('scratch', '?'):>4}  occ {r.get('occ', '?')}  {name[:150]}")

if __name__ == '__main__':
    main(sys.argv[1])
