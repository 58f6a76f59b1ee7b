"""Per-basic-block instruction census of one kernel in a hipcc --save-temps .s file (loop-body
health check: MFMA / ds_read / LDS-DMA / accvgpr-move / waitcnt counts per block).

    python tools/isa_blocks.py file.s kernel_substring
"""
import re
import sys
from collections import Counter

KEYS = ('v_mfma', 'ds_read', 'ds_write', 'global_load', 'global_store', 'v_accvgpr', 's_barrier', 's_waitcnt',
        's_cbranch', 'scratch', 'buffer_')


def main() -> None:
    s = open(sys.argv[1]).read()
    names = re.findall(r'^(\S+):\s*(?:;.*)?$', s, re.M)
    name = next(n for n in names if sys.argv[2] in n and not n.startswith('.'))
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    cur, c, order, blocks = 'entry', Counter(), [], {}
    for line in s[i + len(name) + 1:j].split('\n'):
        t = line.strip()
        m = re.match(r'^(\.LBB\S+):', t)
        if m:
            blocks[cur] = c
            order.append(cur)
            cur, c = m.group(1), Counter()
            continue
        if not t or t.startswith(';') or t.startswith('.'):
            continue
        op = t.split()[0]
        c['n'] += 1
        for k in KEYS:
            if op.startswith(k):
                c[k] += 1
        if op.startswith('s_cbranch') or op.startswith('s_branch'):
            c['->' + t.split()[-1]] += 1
    blocks[cur] = c
    order.append(cur)
    print(name)
    for b in order:
        print(b, dict(blocks[b]))


if __name__ == '__main__':
    main()
