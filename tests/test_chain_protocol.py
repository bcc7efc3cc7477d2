"""A model check of the batch chain's round-flag protocol (ksim_chain.h
chain_block), the race fixed in commit 76f29c9.

Every round of the chain's relaxation, each pod (thread) that changed its
guess lowers a shared "first changed pod" flag; after a barrier every wave
reads the flag and leaves the loop when nothing changed.  The flag must be
reset for the next round.  The pre-76f29c9 code reset its single flag at the
TOP of a round; a wave that is still about to read the previous round's flag
(after the last barrier) then reads the reset value and leaves the loop early.
The fix keeps one flag per round parity and resets the other parity's slot
after the round's first barrier, when every wave has read it.

The model runs waves as sequences of segments between barriers (a barrier
releases when every wave has arrived; between barriers a wave's segment runs
atomically) under chosen interleavings: after each barrier, the segments run
in a given wave order.  The adversarial order (thread 0's wave first, the
reading wave last) is the one the KSIM_CHAIN_DELAY build forces on the device
(tests/test_gpu_chain_race.py)."""
import itertools

import pytest

NONE = 1 << 30


def run(protocol: str, changes, order, n_waves: int):
    """changes[r]: the set of waves with a changed guess in round r (the model
    ignores which pods inside a wave).  Returns each wave's exit round.
    Segments between barriers: 0 = kernel start .. barrier A (round 0's top),
    1 = A .. B, 2 = B .. C, 3 = C .. the next round's A (read the round's
    flag, leave or run the next round's top)."""
    flags = [NONE, NONE]
    exit_round = [None] * n_waves
    rnd = [0] * n_waves
    seg = [0] * n_waves
    done = [False] * n_waves

    def top(w):                                      # the top of a round, before barrier A
        if protocol == "old" and w == 0:
            flags[0] = NONE                          # the single flag, reset at the top

    def segment(w):
        r = rnd[w]
        par = r & 1
        s = seg[w]
        if s == 0:
            top(w)
        elif s == 1:                                 # A .. B
            if protocol == "new" and w == 0:
                flags[par ^ 1] = NONE                # the other parity's slot, after barrier A
        elif s == 2:                                 # B .. C: report a change
            slot = 0 if protocol == "old" else par
            if r < len(changes) and w in changes[r]:
                flags[slot] = min(flags[slot], w)
        else:                                        # C .. next A: read the flag
            slot = 0 if protocol == "old" else par
            if flags[slot] == NONE:
                exit_round[w] = r
                done[w] = True
                return
            rnd[w] += 1
            top(w)
            seg[w] = 1
            return
        seg[w] = s + 1

    guard = 0
    while not all(done):
        # every live wave runs its segment up to the next barrier, in `order`
        for w in [w for w in order if not done[w]]:
            segment(w)
        guard += 1
        assert guard < 1000
    return exit_round


def _expected(changes):
    for r, c in enumerate(changes):
        if not c:
            return r
    return len(changes)


ADVERSARIAL = [0, 1, 2]      # thread 0's wave first, the reading wave (2) last


def test_old_protocol_fails_under_the_adversarial_order():
    changes = [{2}, {1}, set()]                      # two rounds with changes, then a fixpoint
    ex = run("old", changes, ADVERSARIAL, 3)
    assert ex != [_expected(changes)] * 3, "the model must expose the pre-76f29c9 race"


@pytest.mark.parametrize("changes", [[set()], [{0}, set()], [{2}, {1}, set()], [{1, 2}, {0}, {2}, set()],
                                     [{2}, {2}, {2}, {2}, set()]])
def test_per_parity_flags_hold_under_every_order(changes):
    for order in itertools.permutations(range(3)):
        assert run("new", changes, list(order), 3) == [_expected(changes)] * 3, order
