"""Worker for tests/test_distributed.py::test_heartbeat_reports_hung_rank:
rank 1 freezes (SIGSTOP: every thread stops, its sockets stay open, so the
collective transport sees nothing wrong) while rank 0 waits in an
all-reduce; rank 0's heartbeat must name rank 1 and end the process long
before the collective timeout."""
import os
import signal
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from h2o3_amd.parallel import cloud
    cloud.init(device="cpu", timeout_s=1800.0)
    if cloud.rank() == 1:
        time.sleep(1.0)
        os.kill(os.getpid(), signal.SIGSTOP)
    t = torch.ones(4)
    dist.all_reduce(t)      # never completes: the peer is frozen
    print("unexpected: all_reduce returned", t.tolist())


if __name__ == "__main__":
    main()
