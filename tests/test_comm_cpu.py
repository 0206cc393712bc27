"""All-reduce transport thresholds (parallel/comm.py comm_thresholds, the decision part of autotune_comm) from
synthetic timing tables, no GPU."""

from k8s_llm_scheduler_amd.parallel.comm import comm_thresholds

KIB, MIB = 1024, 1 << 20


def test_typical_mi355x_shape():
    # LL wins small messages, two-shot wins from 1 MiB, RCCL wins only past the largest measured size
    table = {16 * KIB: {"ll": 6.0, "oneshot": 8.0, "twoshot": 11.0, "rccl": 25.0},
             64 * KIB: {"ll": 9.0, "oneshot": 10.0, "twoshot": 13.0, "rccl": 28.0},
             256 * KIB: {"ll": 30.0, "oneshot": 19.0, "twoshot": 20.0, "rccl": 35.0},
             1 * MIB: {"oneshot": 60.0, "twoshot": 40.0, "rccl": 55.0},
             4 * MIB: {"twoshot": 110.0, "rccl": 120.0}}
    assert comm_thresholds(table, 4 * MIB) == (64 * KIB, 1 * MIB, 4 * MIB)


def test_rccl_wins_large_messages():
    table = {16 * KIB: {"ll": 6.0, "oneshot": 8.0, "twoshot": 11.0, "rccl": 25.0},
             1 * MIB: {"oneshot": 60.0, "twoshot": 70.0, "rccl": 50.0},
             4 * MIB: {"twoshot": 200.0, "rccl": 120.0}}
    ll, two, xmax = comm_thresholds(table, 4 * MIB)
    # two-shot only where the one-shot kernel cannot run at all; xGMI only for the small messages
    assert ll == 16 * KIB and two == 4 * MIB and xmax == 16 * KIB


def test_ties_prefer_ll_and_no_rccl_means_whole_capacity():
    table = {16 * KIB: {"ll": 8.0, "oneshot": 8.0, "twoshot": 8.0},
             64 * KIB: {"ll": 12.0, "oneshot": 10.0, "twoshot": 10.0}}
    assert comm_thresholds(table, 2 * MIB) == (16 * KIB, 0, 2 * MIB)


def test_empty_table():
    assert comm_thresholds({}, MIB) == (0, 0, 0)
