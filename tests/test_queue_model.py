"""CPU model of the work queue's claim protocol in pair mode (kernels.hip
k_leaf_queue_pair): pair leaders draw the longest groups [0, P) from ticket
q[3]; front waves draw q[0] over [P, ngroups) and then run on into [0, P);
back waves draw q[1] from the short end down to first_short; every group is
claimed by one atomic exchange.  Under random interleavings of the waves'
draws, every group must be hashed exactly once and every wave must stop.
(The device code is the thing under test on the GPU, tests/test_gpu_parity.py
::test_queue_pair; this pins the ticket arithmetic on CPU.)"""
import random

import pytest


def front_group(t, ngroups, P):
    return P + t if t < ngroups - P else t - (ngroups - P)


def simulate(ngroups, P, first_short, n_pairs, n_fronts, n_backs, seed):
    rng = random.Random(seed)
    q = {0: 0, 1: 0, 3: 0}
    claimed = [0] * ngroups
    done = []

    def pull(k):
        t = q[k]
        q[k] += 1
        return t

    def claim(c):
        old = claimed[c]
        claimed[c] = 1
        return old == 0

    def pair_wave():
        while True:  # the pair phase
            g = None
            while True:
                t = pull(3)
                if t >= P:
                    break
                if claim(t):
                    g = t
                    break
            if g is None:
                break
            done.append(g)
            yield
        yield from single_wave(True)

    def single_wave(front):
        while True:
            t = pull(0 if front else 1)
            if t >= ngroups:
                return
            c = front_group(t, ngroups, P) if front else ngroups - 1 - t
            if not front and c < first_short:
                return
            if claim(c):
                done.append(c)
            yield

    waves = [pair_wave() for _ in range(n_pairs)] + [single_wave(True) for _ in range(n_fronts)] + \
        [single_wave(False) for _ in range(n_backs)]
    steps = 0
    while waves:
        w = rng.choice(waves)
        try:
            next(w)
        except StopIteration:
            waves.remove(w)
        steps += 1
        assert steps < 100 * (ngroups + 10) * 10
    return sorted(done)


@pytest.mark.parametrize("seed", range(40))
def test_every_group_once(seed):
    rng = random.Random(seed)
    ngroups = rng.randint(1, 300)
    first_short = rng.randint(0, ngroups)
    P = min(rng.randint(0, ngroups), first_short)
    n_pairs = rng.randint(0, 5) if P else 0
    n_fronts = rng.randint(1, 6)  # every SIMD has a first wave
    n_backs = rng.randint(0, 10)
    done = simulate(ngroups, P, first_short, n_pairs, n_fronts, n_backs, seed)
    assert done == list(range(ngroups))


def test_front_mapping_is_a_permutation():
    for ngroups in (1, 2, 7, 64):
        for P in range(ngroups + 1):
            assert sorted(front_group(t, ngroups, P) for t in range(ngroups)) == list(range(ngroups))
