"""Helpers for multi-process tests that put several ranks on ONE GPU (test infrastructure).

Round 2 offset each rank's device allocations here, after multi-rank runs on one GPU had
intermittently produced wrong temperatures.  Round 3 attributed that: the engine-free probe
(tools/va_probe.hip, profiles/r03/va_probe.txt) shows that two processes never get identical
device virtual addresses (ASLR) and read no foreign values in 6.9e10 reads, and the multi-rank
tests pass without the offset (3 of 3 runs, profiles/r03/multirank_no_offset.txt).  The effect
came from the table-padding memset on the null stream racing the context's stream, fixed in
round 2 after the offset was introduced.  The offset is gone.
"""
import socket


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
