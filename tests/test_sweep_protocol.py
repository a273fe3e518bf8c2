"""CPU model of the persistent sweeps' tile hand-out (rlnc_kernels.hip rlnc_encode_sweep_kernel and
rlnc_decode_sweep_kernel, DECDS_STATIC_SECOND = 1): workgroup b takes tile b, then b + G; from then on every
loop iteration bumps the launch's tile counter, whose answer g names tile 2G + g; a workgroup stops when its
next tile is past the end; each bumps an exit count on the way out and the last one out zeroes both words
for the next launch that takes the slot. Random interleavings of G workgroups check what the kernels rely
on: every tile handed out exactly once, every next tile strictly past the current one (sweep_guard traps
otherwise), and both counter words zero after the launch. A variant of the protocol (the counter zeroed by
the last grab, profiles/HISTORY.md §8 round 5) was checked with this model before it ran on a device; its first form,
which broke the guard on the decode's exit step, fails `test_broken_exit_step_is_caught`."""
import random

import pytest


def run_sweep(total, G, seed, decode, exit_step=None):
    """one launch; returns (tiles in hand-out order, counter words after it)"""
    rnd = random.Random(seed)
    counter = [0, 0]  # tile counter, exit count
    tiles = []

    def wg(b):
        if b >= total:
            return
        k, kn = b, b + G  # current tile, next tile (static second)
        while True:
            more = kn < total
            yield "grab"
            grab = counter[0]
            counter[0] += 1  # every iteration grabs (the tile after the next)
            tiles.append(k)
            yield "tile"
            if decode and exit_step is not None and not more:
                nxt = exit_step(kn, total)
            else:
                nxt = 2 * G + grab
            assert nxt > kn, ("sweep_guard would trap", kn, nxt)  # kn becomes the current tile
            k, kn = kn, nxt
            if not more:
                break
        yield "exit"
        counter[1] += 1
        if counter[1] == G:  # the last workgroup out
            counter[0] = counter[1] = 0

    live = [wg(b) for b in range(min(G, total))]
    grid = len(live)
    if grid < G:  # the launchers size the grid min(tiles, resident): then no counter at all
        return tiles, [0, 0]
    while live:
        g = rnd.choice(live)
        try:
            next(g)
        except StopIteration:
            live.remove(g)
    return tiles, counter


@pytest.mark.parametrize("decode", [False, True])
@pytest.mark.parametrize("total,G", [(512, 512), (513, 512), (1023, 512), (1024, 512), (4096, 512), (4097, 768),
                                     (26368, 768), (103 * 256, 512)])
def test_every_tile_once_guard_holds_counters_reset(total, G, decode):
    for seed in range(3):
        tiles, counter = run_sweep(total, G, seed, decode)
        assert sorted(tiles) == list(range(total))
        assert counter == [0, 0]


def test_broken_exit_step_is_caught():
    # the first form of the last-grab variant set the decode's exit-step next tile to `total`, which is
    # not past a last tile that is already beyond the end: the guard fires (on the box, a trap, r08x)
    with pytest.raises(AssertionError, match="sweep_guard"):
        for seed in range(5):
            run_sweep(4096, 512, seed, decode=True, exit_step=lambda kn, total: total)
    run_sweep(4096, 512, 0, decode=True, exit_step=lambda kn, total: kn + 1)  # the fixed form holds
