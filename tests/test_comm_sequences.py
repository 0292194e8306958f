"""The communicator-sequence check (vtkrylov.comm.check_sequences) the multi-rank GPU tests
apply to the host-staged transport's logs: the RCCL transport hangs when ranks issue different
collectives or unmatched send/receive pairs, so every log must describe a runnable sequence."""
import pytest

from vtkrylov.comm import check_sequences


def _ring_logs(W, sizes):
    """A halo exchange to both x-neighbours (periodic), then an all-reduce, per rank."""
    logs = []
    for r in range(W):
        s = [0] * W
        rv = [0] * W
        for q in ((r - 1) % W, (r + 1) % W):
            if q != r:
                s[q] += sizes
                rv[q] += sizes
        logs.append([("alltoallv", 8, s, rv), ("allreduce", 67), ("allgather", 8)])
    return logs


@pytest.mark.parametrize("W", [2, 3, 8])
def test_matched_sequences_pass(W):
    assert check_sequences(_ring_logs(W, 1600)) == 3


def test_rank_without_neighbours_takes_part_with_zero_counts():
    logs = _ring_logs(3, 800)
    logs.append([("alltoallv", 8, [0] * 4, [0] * 4), ("allreduce", 67), ("allgather", 8)])
    for lg in logs[:3]:
        lg[0] = ("alltoallv", 8, lg[0][2] + [0], lg[0][3] + [0])
    assert check_sequences(logs) == 3


def test_unmatched_send_fails():
    logs = _ring_logs(4, 800)
    op = logs[1][0]
    logs[1][0] = (op[0], op[1], [c * 2 for c in op[2]], op[3])   # rank 1 sends twice what its peers expect
    with pytest.raises(AssertionError):
        check_sequences(logs)


def test_skipped_exchange_fails():
    """A rank that skips an exchange its neighbours send into (the hazard of skipping a
    zero-count exchange on one side only)."""
    logs = _ring_logs(4, 800)
    logs[2][0] = ("alltoallv", 8, [0] * 4, [0] * 4)
    with pytest.raises(AssertionError):
        check_sequences(logs)


def test_allreduce_count_mismatch_fails():
    """Partial vectors all-reduced with a slab-dependent length (a reducing grid that follows
    the rank's rows) -- what the zero-padding to GMAX prevents."""
    logs = _ring_logs(2, 800)
    logs[1][1] = ("allreduce", 1000)
    with pytest.raises(AssertionError):
        check_sequences(logs)
    logs = _ring_logs(2, 800)
    del logs[0][2]
    with pytest.raises(AssertionError):
        check_sequences(logs)
