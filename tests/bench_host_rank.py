"""One rank of the CPU rehearsal of `bench.py --gpus N` (tests/test_bench_cpu.py):
RANK / WORLD_SIZE / MASTER_* come from the test, the collectives run over gloo,
the operators are tests/bench_host_stub.py, the device calls bench.HostDevice.
Arguments are bench.py's own."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
os.environ["SRCDSP_BENCH_BACKEND"] = "gloo"  # read when bench is imported
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import bench  # noqa: E402
import bench_host_stub  # noqa: E402

if __name__ == "__main__":
    bench.main(sys.argv[1:], S=bench_host_stub, dev=bench.HostDevice())
