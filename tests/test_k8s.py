"""Kubernetes cloud formation (h2o3_amd.parallel.k8s): the reference h2o-k8s
lookup contract (H2O_KUBERNETES_SERVICE_DNS / H2O_NODE_EXPECTED_COUNT /
H2O_NODE_LOOKUP_TIMEOUT, leader probe on /kubernetes/isLeaderNode) mapped onto
a torchrun rendezvous.  DNS is simulated; the launcher runs a stand-in for
torchrun's child."""
import urllib.error
import urllib.request

import pytest

from h2o3_amd.parallel import k8s


class _Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t

    def sleep(self, s):
        self.t += s


def test_lookup_waits_for_expected_pods_in_numeric_order():
    answers = [OSError("NXDOMAIN"), {"10.0.0.10"}, {"10.0.0.10", "10.0.0.9"}, {"10.0.0.10", "10.0.0.9", "10.0.0.2"}]
    calls = []

    def resolver(name):
        calls.append(name)
        a = answers[min(len(calls) - 1, len(answers) - 1)]
        if isinstance(a, Exception):
            raise a
        return a
    clk = _Clock()
    ips = k8s.lookup_nodes("svc.ns.svc.cluster.local", expected=3, resolver=resolver, sleep=clk.sleep, clock=clk)
    assert ips == ["10.0.0.2", "10.0.0.9", "10.0.0.10"]          # numeric, not lexicographic
    assert len(calls) == 4 and calls[0] == "svc.ns.svc.cluster.local"


def test_lookup_timeout_ends_with_the_pods_seen():
    clk = _Clock()
    ips = k8s.lookup_nodes("svc", expected=4, timeout_s=5, resolver=lambda n: {"10.1.0.1"}, sleep=clk.sleep,
                           clock=clk)
    assert ips == ["10.1.0.1"] and clk.t >= 5
    with pytest.raises(ValueError):
        k8s.lookup_nodes("  ", expected=1, resolver=lambda n: set())


def test_plan_and_torchrun_command():
    ips = ["10.0.0.2", "10.0.0.9", "10.0.0.10"]
    plan = k8s.node_plan(ips, "10.0.0.9")
    assert plan == {"nnodes": 3, "node_rank": 1, "master_addr": "10.0.0.2", "leader": False}
    assert k8s.node_plan(ips, "10.0.0.2")["leader"]
    cmd = k8s.torchrun_cmd(plan, 8, ["bench.py", "--gpus", "24"], 29511, python="py")
    assert cmd == ["py", "-m", "torch.distributed.run", "--nnodes=3", "--nproc-per-node=8", "--node-rank=1",
                   "--master-addr=10.0.0.2", "--master-port=29511", "bench.py", "--gpus", "24"]
    with pytest.raises(RuntimeError):
        k8s.node_plan(ips, "10.9.9.9")


def test_leader_probe_endpoint():
    lead = k8s.start_probe_api(True, port=0)
    other = k8s.start_probe_api(False, port=0)
    try:
        url = f"http://127.0.0.1:{lead.server_address[1]}/kubernetes/isLeaderNode"
        assert urllib.request.urlopen(url, timeout=5).status == 200
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{other.server_address[1]}/kubernetes/isLeaderNode", timeout=5)
        assert e.value.code == 404
    finally:
        lead.shutdown()
        other.shutdown()


def test_main_launches_child_with_rendezvous(monkeypatch):
    seen = {}
    monkeypatch.setattr(k8s, "lookup_nodes", lambda svc, exp, to, log=None: ["10.0.0.5", "10.0.0.7"])
    monkeypatch.setattr(k8s, "start_probe_api", lambda leader, port=None: seen.setdefault("leader", leader))
    monkeypatch.setattr(k8s.subprocess, "call", lambda cmd, env=None: seen.setdefault("cmd", cmd) and 0)
    env = {"H2O_KUBERNETES_SERVICE_DNS": "svc", "H2O_NODE_EXPECTED_COUNT": "2", "POD_IP": "10.0.0.7",
           "H2O3_GPUS_PER_POD": "8"}
    assert k8s.main(["--", "job.py", "--x"], env=env) == 0
    assert seen["leader"] is False and "--node-rank=1" in seen["cmd"] and seen["cmd"][-2:] == ["job.py", "--x"]
    assert k8s.is_running_on_kubernetes(env) and not k8s.is_running_on_kubernetes({})
