"""Audit the hand-counted loads of the pair and pipe kernels in the built gfx950 assembly.

    python scripts/asm_audit.py [pair|pipe] [path/to/built.s]

local_train_pair.hip (and local_train_pipe.hip, with the same tags) issues its in-loop loads as inline asm (tagged `; pr-row`, `; pr-idx`,
`; pr-poll`) that hipcc does not track, and names each destination in a `; pr-own <reg>`
statement after the counted wait that retires it (cdna_hip_programming.md 5.7 item 1,
form ii).  Between a load and that statement no other instruction may read, write, copy or
spill the destination registers -- hipcc does not know the data is still in flight.  For
every kernel instance this follows every control-flow path from each load to the `pr-own` of
each destination register (or to an `s_waitcnt vmcnt(0)`) and reports any instruction on the
way that references one.  Exit status 1 on a violation.
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'non-iid-distributed-learning-with-optimal-mixture-weights_amd', 'csrc')
KERNELS = {'pair': ('local_train_pair.hip', r'^_Z\w*local_train_pair_kernel\w*:'),
           'pipe': ('local_train_pipe.hip', r'^_Z\w*local_train_pipe_kernel\w*:'),
           'dbuf': ('local_train_dbuf.hip', r'^_Z\w*local_train_dbuf_kernel\w*:')}
REG = re.compile(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b')


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def cfg(lines):
    """Basic blocks of one function: (start, end) line ranges and successor lists."""
    starts = {0}
    labels = {}
    for i, l in enumerate(lines):
        t = l.strip()
        m = re.match(r'^(\.L\w+):', l)
        if m:
            labels[m.group(1)] = i
            starts.add(i)
        elif re.match(r'^; %bb\.\d+:', l):
            starts.add(i)
        op = t.split(';')[0].strip()
        if op.startswith(('s_branch', 's_cbranch', 's_endpgm', 's_setpc')):
            starts.add(i + 1)
    starts = sorted(x for x in starts if x < len(lines))
    blocks = {}
    for k, st in enumerate(starts):
        en = starts[k + 1] if k + 1 < len(starts) else len(lines)
        succ = []
        last = ''
        for i in range(en - 1, st - 1, -1):
            op = lines[i].split(';')[0].strip()
            if op:
                last = op
                break
        m = re.match(r'^s_(c?branch)\w*\s+(\.L\w+)', last)
        if m:
            succ.append(labels[m.group(2)])
            if m.group(1) == 'cbranch' and en < len(lines):
                succ.append(en)
        elif not last.startswith(('s_endpgm', 's_setpc')) and en < len(lines):
            succ.append(en)
        blocks[st] = (en, succ)
    return blocks


def audit_function(name, lines):
    """Every path from each counted load to the `pr-own` of its destinations (or to an
    `s_waitcnt vmcnt(0)`, after which the data has landed) must leave them untouched."""
    blocks = cfg(lines)
    bstart = sorted(blocks)
    import bisect

    def block_of(i):
        return bstart[bisect.bisect_right(bstart, i) - 1]

    bad = 0
    n = 0
    for i, l in enumerate(lines):
        if not re.search(r'; pr-(row|idx|poll)\s*$', l):
            continue
        n += 1
        dest = frozenset(regs(l.split(',')[0]))
        seen = set()
        stack = [(i + 1, dest)]
        while stack:
            pos, pending = stack.pop()
            b = block_of(pos) if pos < len(lines) else None
            if b is None:
                continue
            key = (pos, pending)
            if key in seen:
                continue
            seen.add(key)
            en, succ = blocks[b]
            k = pos
            while k < en and pending:
                t = lines[k]
                op = t.split(';')[0].strip()
                if '; pr-own' in t:
                    pending = pending - regs(t.split('pr-own', 1)[1])
                elif op.startswith('s_waitcnt') and re.search(r'vmcnt\(0\)', op):
                    pending = frozenset()
                elif op and not op.startswith('s_waitcnt'):
                    hit = regs(op) & pending
                    is_load = re.search(r'; pr-(row|idx|poll)', t)
                    if hit and not (is_load and not (regs(op.split(',')[0]) & pending)):
                        print('%s: line %d (load at %d: %s) touches v%s in flight:\n    %s' %
                              (name[:60], k, i, l.strip()[:60], sorted(hit), t.strip()[:100]))
                        bad += 1
                        pending = pending - hit
                    elif hit and is_load:
                        pending = pending - hit          # a new counted load into the same register
                k += 1
            if pending:
                for sb in succ:
                    stack.append((sb, pending))
    return n, bad


def main():
    args = sys.argv[1:]
    kind = args.pop(0) if args and args[0] in KERNELS else 'pair'
    src, fre = KERNELS[kind]
    path = args[0] if args else '/tmp/local_train_%s.s' % kind
    if not args:
        subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950',
                               '-munsafe-fp-atomics', '--cuda-device-only', '-S', os.path.join(CSRC, src), '-o', path])
    text = open(path).read().split('\n')
    funcs = [(i, l.split(':')[0]) for i, l in enumerate(text) if re.match(fre, l)]
    total_bad = total = 0
    for fi, (start, name) in enumerate(funcs):
        end = next(i for i in range(start, len(text)) if text[i].startswith('.Lfunc_end'))
        n, bad = audit_function(name, text[start:end])
        total += n
        total_bad += bad
        print('%-70s %3d counted loads, %d violations' % (name[:70], n, bad))
    sys.exit(1 if total_bad else 0)


if __name__ == '__main__':
    main()
