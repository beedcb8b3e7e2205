"""CPU model of the grid decode's phase-F vocabulary schedule (decode_grid.hip phase_f): the
static blocks w + G (FSL u + k), the claimed chunks of FSL consecutive blocks from
d0 = G FSL su (claimed three outer iterations ahead, published through a 4-entry LDS ring), and
the loop bounds -- restated index for index from the kernel, with the workgroups interleaved in
random orders and at random relative speeds.  Asserts: every vocabulary block is consumed exactly
once, every ring entry read is the one published for that iteration, in both the persistent
(claims) and the phase-launch (static) forms, for every grid size and for vocabularies from the
kernel's minimum (16 G 3 ids) to GPT-2's.  (A static-form bound that went negative once left a
row without any block -- an argmax key nobody raised; this is the check that would have said so
on the CPU.)
"""
import random

import pytest

NSL = 4          # Geo<G>::FSL


def schedule(G, V, dyn_wanted, seed):
    nvb = (V + 15) >> 4
    su = (nvb + G * NSL - 1) // (G * NSL)
    dyn = False
    if dyn_wanted:
        s2 = max(3, (nvb * 5 // 8) // (G * NSL))
        if G * NSL * s2 <= nvb - G:
            su, dyn = s2, True
    d0 = G * NSL * su
    nch = (nvb - d0 + NSL - 1) // NSL if dyn else 0
    counter = [0]
    seen = [0] * nvb
    rng = random.Random(seed)

    def wg(w):
        chr_ = [None] * 4
        pend = None

        def iter_blocks(u):
            if u < su:
                return w + G * NSL * u, G
            if dyn:
                tag, c = chr_[u & 3]
                assert tag == u, f"ring entry of iteration {tag} read for {u}"
                return d0 + NSL * c, 1
            return 0x3FFFFFFF, 0

        bu, stu = iter_blocks(0)
        u = 0
        while bu < nvb and u < su + nch:
            bn, stn = iter_blocks(u + 1) if (u + 1 < su or not dyn or chr_[(u + 1) & 3] is not None
                                              and chr_[(u + 1) & 3][0] == u + 1) else (None, None)
            for k in range(NSL):
                b = bu + k * stu
                if b < nvb:
                    seen[b] += 1
                if k == 1 and dyn and u >= su - 3:
                    if u >= su - 2:
                        chr_[(u + 2) & 3] = (u + 2, pend)
                    pend = counter[0]
                    counter[0] += 1
                    yield           # other workgroups run between this claim and the next
            assert bn is not None, f"iteration {u + 1}'s chunk read before it was published"
            bu, stu = bn, stn
            u += 1
            yield

    gens = [wg(w) for w in range(G)]
    speed = [rng.choice([1, 1, 1, 2, 3]) for _ in range(G)]
    live = list(range(G))
    while live:
        w = rng.choice(live)
        try:
            for _ in range(speed[w]):
                next(gens[w])
        except StopIteration:
            live.remove(w)
    return seen, dyn


@pytest.mark.parametrize("G", [48, 96, 192])
@pytest.mark.parametrize("V", [50257, 16 * 48 * 3, 16 * 192 * 3, 12345, 16 * 192 * 13 + 7])
@pytest.mark.parametrize("dyn", [True, False])
def test_every_vocab_block_once(G, V, dyn):
    if V < 16 * G * 3:
        pytest.skip("below the kernel's minimum vocabulary for this grid (dg_args)")
    for seed in range(3):
        seen, used_dyn = schedule(G, V, dyn, seed)
        bad = [b for b, n in enumerate(seen) if n != 1]
        assert not bad, f"G {G} V {V} dyn {used_dyn}: blocks consumed != once: {bad[:8]}"


def test_gpt2_vocab_takes_the_claims():
    for G in (48, 96, 192):
        assert schedule(G, 50257, True, 0)[1], f"G {G}: GPT-2's vocabulary should use claims"
