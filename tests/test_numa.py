"""Host NUMA placement helper (rdfind_amd/numa.py): cpulist parsing and the no-GPU / unknown-topology path."""
import os

from rdfind_amd import numa


def test_parse_cpulist():
    assert numa._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa._parse_cpulist("5") == {5}
    assert numa._parse_cpulist("") == set()


def test_bind_without_a_gpu_changes_nothing():
    before = os.sched_getaffinity(0)
    node = numa.bind_to_device_node(0)  # no GPU here: the node is unknown
    if node is None:
        assert os.sched_getaffinity(0) == before
    else:  # (a GPU host) bound to that node's CPUs
        assert os.sched_getaffinity(0) <= before
