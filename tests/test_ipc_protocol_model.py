"""CPU model of the IPC halo signalling protocol (kernels/ipc_flags.hip,
src/ipc_halo.cpp): push-to-the-poller mailboxes.

Per exchange n, each rank (thread 0 of its dispatch) stores "my rows are
final" into its neighbours' mailboxes (its upper neighbour's `level_down`,
its lower neighbour's `level_up`), waits for its own `level_up` /
`level_down`, pulls, then acks the same way (`ack_down` / `ack_up`) before
`count` advances.  Which mailbox a rank signals is decided on the host
(IpcHaloTransport::exchange): the neighbours' for real ranks; for a
self-neighbour (the one-process emulation of a rank, bench.py --emulate
W:R --emulate-halo ipc) its own mailbox on BOTH sides — an emulated edge
band has one neighbour, itself, and with the neighbour-side rule alone its
one-sided wait read a word nobody stored (it timed out on the GPU).

The model runs every rank's sequence of stores and bounded waits under all
interleavings a round-robin scheduler produces and checks that each
exchange completes; the GPU tests (tests/test_gpu_ipc.py) check the kernels.
"""
import itertools

import pytest


class Mailbox:
    def __init__(self):
        self.level_up = self.level_down = self.ack_up = self.ack_down = self.count = 0


def exchange_program(mine, up_mb, down_mb, n):
    """The kernel's signal / wait / ack sequence for exchange n as a
    generator: yields a predicate while waiting, performs stores inline."""
    if up_mb is not None:
        up_mb.level_down = n  # I am my upper neighbour's lower neighbour
    if down_mb is not None:
        down_mb.level_up = n
    if up_mb is not None:
        while mine.level_up < n:
            yield
    if down_mb is not None:
        while mine.level_down < n:
            yield
    # (pull of the neighbours' rows here)
    mine.count = n
    if up_mb is not None:
        up_mb.ack_down = n
    if down_mb is not None:
        down_mb.ack_up = n
    if up_mb is not None:
        while mine.ack_up < n:
            yield
    if down_mb is not None:
        while mine.ack_down < n:
            yield


def mailboxes_for(bands, boxes, self_rule):
    """(mine, up_mb, down_mb) per rank as IpcHaloTransport::exchange passes
    them.  bands[r] = (up, down) rank indices or None; a band whose
    neighbour is itself is the emulation's self-neighbour."""
    out = []
    for r, (up, down) in enumerate(bands):
        own = up == r or down == r
        if own and self_rule == "both":
            out.append((boxes[r], boxes[r], boxes[r]))
        else:
            out.append((boxes[r], boxes[up] if up is not None else None, boxes[down] if down is not None else None))
    return out


def run(bands, exchanges=3, self_rule="both", order=None, budget=10_000):
    boxes = [Mailbox() for _ in bands]
    args = mailboxes_for(bands, boxes, self_rule)
    for n in range(1, exchanges + 1):
        progs = [exchange_program(*a, n) for a in args]
        live = list(range(len(progs)))
        steps = 0
        seq = itertools.cycle(order or range(len(progs)))
        while live:
            r = next(seq)
            if r not in live:
                continue
            try:
                next(progs[r])
            except StopIteration:
                live.remove(r)
            steps += 1
            if steps > budget:
                return False  # a wait that nobody satisfies: the GPU's bounded wait times out
    return all(b.count == exchanges for b in boxes)


def chain(world):
    return [(r - 1 if r > 0 else None, r + 1 if r < world - 1 else None) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("order", ["forward", "reverse"])
def test_real_ranks_complete(world, order):
    o = list(range(world)) if order == "forward" else list(reversed(range(world)))
    assert run(chain(world), order=o)


@pytest.mark.parametrize("band", [(0, 0), (None, 0), (0, None)])
def test_self_neighbour_completes_with_both_sides(band):
    """An emulated interior band (itself above and below) and an emulated
    edge band (itself on one side only) both complete."""
    assert run([band])


def test_one_sided_self_neighbour_needs_both_sides():
    """The first rule (only the existing side signalled) deadlocks for an
    emulated edge band — the GPU run of bench.py --emulate 2:0 timed out."""
    assert not run([(None, 0)], self_rule="sides")
    assert not run([(0, None)], self_rule="sides")
    assert run([(0, 0)], self_rule="sides")  # the interior emulation worked either way
