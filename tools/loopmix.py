"""Instruction mix of a kernel's outer loop body in a hipcc -S listing (static counts):
    python tools/loopmix.py build/vtk_band.s _ZN3vtk11k_band_stepILi5ELi18ELi2ELi2EEEvNS_5BandKE"""
import re
import sys
from collections import Counter


def mix(path, name):
    lines, on = [], False
    for l in open(path):
        l = l.rstrip('\n')
        if l.startswith(name + ':'):
            on = True
            continue
        if on and re.match(r'^_Z\w+:', l):
            break
        if on:
            lines.append(l)
    best = (None, Counter())
    for h in [l.split(':')[0][1:] for l in lines if 'Loop Header: Depth=1' in l]:
        c, inloop = Counter(), False
        for l in lines:
            if re.match(r'^(\.LBB|; %bb)', l):
                inloop = l.startswith('.' + h + ':') or re.search(r'Header=' + h[1:] + r'\b', l) is not None
                continue
            if inloop:
                m = re.match(r'\s+([a-z_0-9]+)', l)
                if m:
                    c[m.group(1)] += 1
        if sum(c.values()) > sum(best[1].values()):
            best = (h, c)
    return best


if __name__ == '__main__':
    hdr, c = mix(sys.argv[1], sys.argv[2])
    v = sum(n for k, n in c.items() if k.startswith('v_'))
    s = sum(n for k, n in c.items() if k.startswith('s_'))
    print(hdr, 'VALU', v, 'SALU', s)
    for k, n in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
        print(n, k)
