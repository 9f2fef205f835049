"""Host logic of the pointer-table slot grids (shmr_amd/csrc/ptr_grid.hpp), on
the CPU: tools/ptr_grid_check.cpp is compiled with g++ and fed tables.

A *_ptrs_dev table is run through the strided kernels only when fit_grid finds
(base, block pitch, shard pitch) that reproduce every entry in the kernels'
unsigned 64-bit arithmetic.  Soundness -- a returned grid
reproduces every entry, pitches non-negative -- is what keeps the bytes
identical to the table kernels'; completeness -- every slab-shaped table,
including sparse ones where no block holds two entries (a rebuild of one lost
shard per block), is recognised -- is what keeps the speed.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("grid") / "ptr_grid_check")
    # under ASan + UBSan (any report aborts the checker and fails the test): the
    # solver's __int128 products and its wrapping uint64 reproduction
    subprocess.run(["g++", "-O1", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "shmr_amd", "csrc"),
                    os.path.join(ROOT, "tools", "ptr_grid_check.cpp"), "-o", exe], check=True)

    def run(cases):
        inp = "".join(f"{len(c)}\n" + "".join(f"{b} {j} {a}\n" for b, j, a in c) for c in cases)
        out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
        res = []
        for line in out[:len(cases)]:
            f = line.split()
            res.append(None if f[0] == "0" else tuple(int(x) for x in f[1:]))
        return res
    return run


M64 = (1 << 64) - 1


def _reproduces(case, g):
    base, bp, sp = g
    return all(a == (base + b * bp + j * sp) & M64 for b, j, a in case) and bp >= 0 and sp >= 0


def _grid_case(rng, sparse):
    B = int(rng.integers(1, 9))
    n = int(rng.integers(1, 12))
    sp = int(rng.choice([16, 4096, 528384, int(rng.integers(1, 1 << 21))]))
    bp = n * sp + int(rng.integers(0, 3)) * int(rng.choice([1, 7, 4096]))
    if rng.integers(0, 3) == 0:
        bp = int(rng.integers(0, 4)) * sp          # degenerate strides (collinear / overlapping blocks)
    base = int(rng.integers(1 << 40, 1 << 47))
    case = []
    for b in range(B):
        js = range(n)
        if sparse:
            js = sorted(rng.choice(n, size=int(rng.integers(0, min(n, 2) + 1)), replace=False).tolist())
        for j in js:
            case.append((b, j, base + b * bp + j * sp))
    return case


def test_slab_shaped_tables_fit(checker):
    rng = np.random.default_rng(31)
    cases = [_grid_case(rng, sparse=bool(i % 2)) for i in range(4000)]
    cases = [c for c in cases if c]
    res = checker(cases)
    for c, g in zip(cases, res):
        assert g is not None, c[:6]
        assert _reproduces(c, g)


def test_one_entry_per_block_with_varying_shard(checker):
    """The case a dense-pair-only fit missed (r05 sweep case 217): RS(1,1)
    blocks rebuilding one lost shard each -- no block holds two entries, the
    shard index differs between blocks."""
    sp, bp, base = 4111, 8236, 5
    case = [(0, 0, base), (1, 0, base + bp), (2, 1, base + 2 * bp + sp)]
    g = checker([case])[0]
    assert g == (base, bp, sp)


def test_tables_off_a_grid_are_refused_or_reproduced(checker):
    """Soundness: perturbed and shuffled tables either find no grid or a grid
    that reproduces every entry (then the strided kernels touch exactly the
    table's addresses)."""
    rng = np.random.default_rng(32)
    cases = []
    for _ in range(3000):
        c = _grid_case(rng, sparse=False)
        if len(c) < 2:
            continue
        c = list(c)
        kind = int(rng.integers(0, 3))
        i = int(rng.integers(0, len(c)))
        if kind == 0:                                   # one address off by a few bytes
            b, j, a = c[i]
            c[i] = (b, j, a + int(rng.integers(1, 64)))
        elif kind == 1:                                 # two entries' addresses swapped
            i2 = int(rng.integers(0, len(c)))
            (b1, j1, a1), (b2, j2, a2) = c[i], c[i2]
            c[i], c[i2] = (b1, j1, a2), (b2, j2, a1)
        else:                                           # descending pitch (not a slab)
            c = [(b, j, (1 << 47) - a % (1 << 46)) for b, j, a in c]
        cases.append(c)
    refused = 0
    for c, g in zip(cases, checker(cases)):
        if g is None:
            refused += 1
        else:
            assert _reproduces(c, g), c[:6]
    assert refused > len(cases) // 2


def test_duplicate_position_and_wrapping(checker):
    assert checker([[(0, 0, 4096), (0, 0, 8192)]]) == [None]
    # addresses near the top of the 64-bit space: the grid is checked modulo 2^64
    top = (1 << 64) - 3 * 4096
    g = checker([[(0, 0, top), (0, 1, top + 4096), (1, 0, top + 8192 - 4096 + 4096)]])[0]
    assert g is not None and _reproduces([(0, 0, top), (0, 1, top + 4096), (1, 0, top + 8192)], g)


def test_adversarial_extremes(checker):
    """Entries with addresses anywhere in the 64-bit space, block indices up to
    2^40 and shard indices up to 255, random or on extreme grids: the solver's
    exact-integer steps run under UBSan without a report, and every grid it
    returns reproduces the table."""
    rng = np.random.default_rng(33)
    cases = []
    for i in range(2000):
        n = int(rng.integers(2, 9))
        bs = sorted(set(int(x) for x in rng.integers(0, 1 << 40, size=n)))
        if i % 2:                                   # on a grid with huge pitches, wrapping mod 2^64
            base = int(rng.integers(0, 1 << 63)) * 2
            bp, sp = int(rng.integers(0, 1 << 62)), int(rng.integers(0, 1 << 62))
            case = [(b, int(j), (base + b * bp + int(j) * sp) & M64) for b in bs for j in sorted(
                set(int(x) for x in rng.integers(0, 256, size=2)))]
        else:                                       # random addresses
            case = [(b, int(rng.integers(0, 256)), int(rng.integers(0, 1 << 63)) * 2 + int(rng.integers(0, 2)))
                    for b in bs]
        cases.append(case)
    for c, g in zip(cases, checker(cases)):
        if g is not None:
            assert _reproduces(c, g), c[:4]


# ---- slot lattices (r06): rows in any order, with holes ------------------------------
@pytest.fixture(scope="module")
def lattice(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("lattice") / "lattice_check")
    subprocess.run(["g++", "-O1", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "shmr_amd", "csrc"),
                    os.path.join(ROOT, "tools", "lattice_check.cpp"), "-o", exe], check=True)

    def run(cases):
        """cases: (nrows, entries, entries2) with entries [(row, j, addr)]."""
        inp = "".join(f"{n} {len(e1)} {len(e2)}\n" + "".join(f"{r} {j} {a}\n" for r, j, a in e1 + e2)
                      for n, e1, e2 in cases)
        out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
        res = []
        for (n, _, e2), line in zip(cases, out):
            f = [int(x) for x in line.split()]
            if f[0] == 0:
                res.append(None)
                continue
            g1 = tuple(f[1:4])
            g2 = tuple(f[4:7]) if e2 else None
            res.append((g1, g2, f[7 if e2 else 4:]))
        return res
    return run


def _lattice_ok(entries, g, slots):
    base, bp, sp = g
    return all(a == (base + slots[r] * bp + j * sp) & M64 for r, j, a in entries)


def _pool_case(rng, holes, joint):
    """A pool slab's live blocks in shuffled order: encode inputs (j < k) and
    outputs (j - k), from a joint slot layout or separate data / parity slabs."""
    k, p = int(rng.integers(1, 11)), int(rng.integers(1, 5))
    t = k + p
    P = int(rng.choice([4096, 528384, 1679360, 16 * int(rng.integers(1, 1 << 12))]))
    nslots = int(rng.integers(1, 300))
    live = sorted(rng.choice(nslots, size=max(1, nslots - (int(rng.integers(0, nslots)) if holes else 0)),
                             replace=False).tolist())
    order = rng.permutation(len(live))
    base = int(rng.integers(1 << 40, 1 << 47)) // 256 * 256
    pbase = base + nslots * k * P + int(rng.integers(0, 64)) * 4096
    ins, outs = [], []
    for r, o in enumerate(order):
        s = live[int(o)]
        for i in range(t):
            if joint:
                a = base + s * t * P + i * P
            else:
                a = base + s * k * P + i * P if i < k else pbase + s * p * P + (i - k) * P
            (ins if i < k else outs).append((r, i if i < k else i - k, a))
    return len(live), ins, outs, [live[int(o)] for o in order]


def test_pool_tables_fit_a_lattice(lattice):
    """Completeness: a pool's live blocks in any order, with holes, joint or
    separate data / parity slabs, always fit (inputs; outputs over the same
    slots), and the lattice reproduces every address."""
    rng = np.random.default_rng(61)
    cases, meta = [], []
    for i in range(1500):
        n, ins, outs, live = _pool_case(rng, holes=bool(i % 2), joint=bool(i % 3 == 0))
        cases.append((n, ins, outs))
        meta.append(live)
    for (n, ins, outs), res, live in zip(cases, lattice(cases), meta):
        assert res is not None, (n, ins[:4])
        g1, g2, slots = res
        assert _lattice_ok(ins, g1, slots) and _lattice_ok(outs, g2, slots)
        assert len(set(slots)) == n and max(slots) < (1 << 32)
        # the slots keep the pool's order (a lattice may be coarser, never reordered)
        assert np.array_equal(np.argsort(slots, kind="stable"), np.argsort(live, kind="stable"))


def test_off_lattice_tables_refused_or_reproduced(lattice):
    """Soundness: perturbed, duplicated or swapped rows either find no lattice
    or one that reproduces every entry; duplicate rows (one slot twice) are
    always refused."""
    rng = np.random.default_rng(62)
    cases = []
    for i in range(2000):
        n, ins, outs, _ = _pool_case(rng, holes=True, joint=bool(i % 2))
        ins, outs = list(ins), list(outs)
        kind = i % 4
        if kind == 0:
            q = int(rng.integers(0, len(ins)))
            r, j, a = ins[q]
            ins[q] = (r, j, a + int(rng.integers(1, 4096)))
        elif kind == 1:
            q = int(rng.integers(0, len(outs)))
            r, j, a = outs[q]
            outs[q] = (r, j, a - int(rng.integers(1, 64)))
        elif kind == 2 and n > 1:   # row 1 names row 0's block: the same slot twice
            ins = [(r, j, a) for r, j, a in ins if r != 1] + [(1, j, a) for r, j, a in ins if r == 0]
            ins.sort()
        cases.append((n, ins, outs))
    refused = 0
    for (n, ins, outs), res in zip(cases, lattice(cases)):
        if res is None:
            refused += 1
            continue
        g1, g2, slots = res
        assert _lattice_ok(ins, g1, slots) and _lattice_ok(outs, g2, slots)
        assert len(set(slots)) == n
    assert refused > len(cases) // 2


def test_lattice_single_rows_and_wrapping(lattice):
    # one row, one entry: any address is a lattice of one slot (pitches 0)
    assert lattice([(1, [(0, 3, 12345)], [])]) == [((12345, 0, 0), None, [0])]
    # rows that each touch one shard (a rebuild of one lost shard per block)
    res = lattice([(3, [(0, 2, 100 + 2 * 7), (1, 0, 100 + 50), (2, 1, 100 + 100 + 7)], [])])[0]
    assert res is not None and _lattice_ok([(0, 2, 114), (1, 0, 150), (2, 1, 207)], res[0], res[2])
    # descending shard pitch inside a row is refused (not a slot layout)
    assert lattice([(1, [(0, 0, 8192), (0, 1, 4096)], [])]) == [None]
