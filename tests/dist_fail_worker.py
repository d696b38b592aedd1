"""Worker for tests/test_distributed.py::test_failed_rank_exits_fast: rank 1
raises while rank 0 waits in an all-reduce; the exit-time teardown of the
failed rank must not sit in a barrier (parallel/cloud.py shutdown)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from h2o3_amd.parallel import cloud
    cloud.init(device="cpu", timeout_s=1800.0)
    if cloud.rank() == 1:
        raise RuntimeError("simulated failure on rank 1")
    t = torch.ones(4)
    dist.all_reduce(t)      # never completes normally: the peer is gone
    print("unexpected: all_reduce returned", t.tolist())


if __name__ == "__main__":
    main()
