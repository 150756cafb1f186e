"""§8f.3/.4 on the GPU: the HBM-resident FifoWithTimeTrack replays every golden
script recorded from the real reference (buffers.h), through host and device
write/read paths; a producer thread and a consumer thread stream through it
concurrently; binary I/Q captures load into and save from device memory with
the reference's bytes (dsptl_files.h)."""
import threading

import numpy as np
import pytest

from io_replay import load, replay_fifo, elem_dtype

pytestmark = pytest.mark.gpu
MAN, ARR = load()


class _HostAdapter:
    def __init__(self, f):
        self.f = f
        self.write = f.write
        self.count = f.count
        self.reset = f.reset

    def read(self, n, start):
        return self.f.read(n, start)

    def absolute_time(self, tp, frac):
        return self.f.getAbsoluteTime(tp, frac)


class _DeviceAdapter(_HostAdapter):
    """writes and reads through device (torch) buffers"""

    def __init__(self, f, dt):
        super().__init__(f)
        self.dt = dt
        import torch
        self.torch = torch
        self.write = self._write

    def _write(self, x, sec, frac):
        t = self.torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1)).cuda()
        self.f.write(t, sec, frac)

    def read(self, n, start):
        out = self.torch.zeros(n * self.dt.itemsize, dtype=self.torch.uint8, device="cuda")
        err, st, out = self.f.read(out, start)
        return err, st, out.cpu().numpy()


@pytest.mark.parametrize("path", ["host", "device"])
@pytest.mark.parametrize("case", MAN["fifo"], ids=[c["name"] for c in MAN["fifo"]])
def test_fifo_replays_reference_scripts(S, case, path):
    dt = elem_dtype(case)
    f = S.FifoWithTimeTrack(dt, case["N"], case["fs"])
    replay_fifo(_HostAdapter(f) if path == "host" else _DeviceAdapter(f, dt), case, ARR)


def test_fifo_errors(S):
    from srcdsp_amd._capi import ERR_SIZE, SrcdspError
    f = S.FifoWithTimeTrack(np.int32, 16)
    with pytest.raises(SrcdspError) as e:
        f.write(np.zeros(16, np.int32))  # assert(inSize < N)
    assert e.value.code == ERR_SIZE
    with pytest.raises(SrcdspError) as e:
        f.read(0, 1)  # assert(out.size() != 0)
    assert e.value.code == ERR_SIZE


def test_fifo_concurrent_producer_consumer(S):
    """SPSC streaming: the producer writes 300 blocks (host path, double
    buffered) while the consumer reads recent ranges into device memory; every
    value read equals the function of its time index that was written."""
    import torch
    N, B, blocks = 1 << 20, 10000, 300
    f = S.FifoWithTimeTrack(np.int32, N, 1e6)

    def val(t):
        return ((t * 2654435761) & 0x7FFFFFFF).astype(np.int32)

    errors = []

    def producer():
        try:
            for b in range(blocks):
                t = np.arange(b * B + 1, (b + 1) * B + 1, dtype=np.int64)
                f.write(val(t), b, 0.0)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = threading.Thread(target=producer)
    th.start()
    checked = 0
    out = torch.empty(4096, dtype=torch.int32, device="cuda")
    while th.is_alive() or checked < 50:
        wp, ts, te, _ = f.state()
        if te < 8192 + 4096:
            continue
        start = te - 4096 - 4096  # well behind the writer, inside the ring
        err, st, o = f.read(out, start)
        assert not err and st == start
        t = np.arange(start, start + 4096, dtype=np.int64)
        assert np.array_equal(o.cpu().numpy(), val(t)), start
        checked += 1
        if not th.is_alive() and checked >= 50:
            break
    th.join()
    assert not errors
    assert f.count() == N  # full ring: timeEnd - timeStart + 1


@pytest.mark.parametrize("case", MAN["iq"], ids=[c["name"] for c in MAN["iq"]])
def test_iq_device_load_and_save(S, case, tmp_path):
    import torch
    from srcdsp_amd import files
    x = ARR[case["samples"]]
    path = str(tmp_path / "cap.bin")
    with open(path, "wb") as fh:
        fh.write(ARR[case["file"]].tobytes())  # the reference's bytes
    d = files.readBinarySamples(path, x.dtype, device=True)
    assert d.is_cuda and np.array_equal(d.cpu().numpy(), x)
    out = str(tmp_path / "back.bin")
    files.saveBinarySamples(d, out)
    with open(out, "rb") as fh:
        assert fh.read() == ARR[case["file"]].tobytes()
    del torch


def test_iq_device_large_multi_chunk(S, tmp_path):
    """> 2 staging chunks each way (8 MiB chunks): 40 MiB of complex<float>."""
    import torch
    from srcdsp_amd import files
    n = 5 << 20
    x = torch.randn((n, 2), dtype=torch.float32, device="cuda")
    p = str(tmp_path / "big.bin")
    files.saveBinarySamples(x, p)
    assert files.countBinarySamples(p, "complex<float>") == n
    y = files.readBinarySamples(p, "complex<float>", device=True)
    assert torch.equal(x, y)
