"""CPU replay of the hash kernels' rank commit (include/combblas_hip/device/task_kernel.h:
queue_run_start + rank_commit_batch) on random occupancy patterns: the occupied
slots of an order-preserving table form runs whose keys are unordered inside a run and ordered
between runs; every wave takes a queue range cut at run starts and commits it in batches of <= 64
entries that end where a run starts, ranking each key among its run's keys by lane shuffles (LDS
walks only for runs longer than a batch or a wave edge with no run start within 64 entries).
The replay follows the kernel's lane arithmetic (ballot masks, clz/ffs, the batch limit) and must
place every key exactly where a sort puts it -- fills up to 0.95 exercise the long-run fallbacks."""
import numpy as np
import pytest

M64 = (1 << 64) - 1


def _clz(x):
    return 64 - int(x).bit_length()


def _ffs(x):
    return (x & -x).bit_length()


def _queue_run_start(Q, nom):
    qtot = len(Q)
    if nom <= 0:
        return 0
    if nom >= qtot:
        return qtot
    m = 0
    for lane in range(64):
        x = nom + lane
        if x >= qtot or Q[x] != Q[x - 1] + 1:
            m |= 1 << lane
    return nom + _ffs(m) - 1 if m else nom


def _commit(Q, keys, NW):
    """output position of every queue entry, as the NW waves of one workgroup compute them"""
    qtot = len(Q)
    out = [None] * qtot
    per = (qtot + NW - 1) // NW
    for w in range(NW):
        qs = _queue_run_start(Q, w * per)
        qe = qtot if w == NW - 1 else _queue_run_start(Q, (w + 1) * per)
        b0 = qs
        while b0 < qe:
            loaded = [b0 + l < qtot for l in range(64)]
            sq = [Q[b0 + l] if loaded[l] else -4 for l in range(64)]
            key = [keys[sq[l]] if loaded[l] else 2**31 - 1 for l in range(64)]
            sprev = [(Q[b0 - 1] if b0 > 0 else -10) if l == 0 else sq[l - 1] for l in range(64)]
            snext = [(Q[b0 + 64] if l == 63 else sq[l + 1]) if b0 + l + 1 < qtot else -10 for l in range(64)]
            mstart = sum(1 << l for l in range(64) if loaded[l] and sq[l] != sprev[l] + 1)
            mend = sum(1 << l for l in range(64) if loaded[l] and snext[l] != sq[l] + 1)
            limit = 64
            if b0 + 64 <= qe and not (mend >> 63) & 1 and mstart:
                last = 63 - _clz(mstart)
                if last > 0:
                    limit = last
            used = min(qe - b0, limit)
            for l in range(64):
                if not (b0 + l < qe and l < limit):
                    continue
                below = mstart & (M64 if l == 63 else (2 << l) - 1)
                above = mend & ~((1 << l) - 1) & M64
                rs = 63 - _clz(below) if below else -1
                re = _ffs(above) - 1 if above else 64
                lo, hi = max(rs, 0), min(re, 63)
                rank = sum(1 for j in range(lo, hi + 1) if key[j] < key[l])
                rstart = b0 + lo
                if rs < 0:
                    qq = b0 - 1
                    while qq >= 0 and Q[qq] == Q[qq + 1] - 1:
                        rank += keys[Q[qq]] < key[l]
                        qq -= 1
                    rstart = qq + 1
                if re > 63:
                    qq = b0 + 64
                    while qq < qtot and Q[qq] == Q[qq - 1] + 1:
                        rank += keys[Q[qq]] < key[l]
                        qq += 1
                out[b0 + l] = rstart + rank
            b0 += used
    return out


@pytest.mark.parametrize("seed", range(4))
def test_rank_commit_places_every_key_in_sorted_order(seed):
    rng = np.random.default_rng(seed)
    for _ in range(60):
        T = int(rng.integers(64, 2200))
        occ = rng.random(T) < rng.uniform(0.2, 0.95)
        Q = [int(x) for x in np.nonzero(occ)[0]]
        if not Q:
            continue
        keys, base, run = {}, 0, [Q[0]]
        for a, b in zip(Q, Q[1:] + [None]):
            if b is not None and b == a + 1:
                run.append(b)
                continue
            for s, p in zip(run, rng.permutation(len(run))):  # unordered inside a run
                keys[s] = base + int(p)
            base += len(run)
            run = [b]
        out = _commit(Q, keys, int(rng.choice([1, 2, 4, 8])))
        assert sorted(out) == list(range(len(Q)))
        assert all(keys[Q[i]] == out[i] for i in range(len(Q)))
