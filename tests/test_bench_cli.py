"""bench.py's command line outside a launcher: `python bench.py --gpus N` (N > 1) with no
torch.distributed environment starts itself under torch.distributed.run as a child process (one
rank per GPU, rendezvous on 127.0.0.1, the same arguments) and exits with the child's code."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_without_launcher_starts_torchrun_child(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "8", "--warmup", "2"])
    assert bench.main() == 7
    (cmd,) = calls
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert any(c.startswith("--master-port=") for c in cmd)
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "8", "--warmup", "2"]


def test_traffic_counts_the_product_kernels_only():
    """The HBM traffic pass sums the uninstrumented tracescreen launch: the STATS instantiations are
    recognised by their template argument (k_trace<L, STATS>, k_camerarays_group<STATS, ...>), not by
    the word `true` anywhere in the name."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.instrumented_kernel("k_trace<0, true>")
    assert bench.instrumented_kernel("k_trace<3, true>")
    assert bench.instrumented_kernel("k_camerarays_group<true, 512, 8>")
    assert not bench.instrumented_kernel("k_trace<0, false>")
    assert not bench.instrumented_kernel("k_trace<0, false, true>")  # a later template flag is not STATS
    assert not bench.instrumented_kernel("k_camerarays_group<false, 512, 4>")
    assert not bench.instrumented_kernel("k_finish")
