#!/usr/bin/env python3
"""Benchmark of the SrcDsp hot path on MI355X (driver contract: one JSON line).

Default workload = BASELINE.json configs[1] (the headline metric): the 127-tap
complex<float> decimate-by-4 FilterDnsamplingFir over 2^28 device-resident
synthetic samples, one step() per timed step (one kernel launch), FMA float
contract.  With --gpus N (launched by torch.distributed.run) every rank owns
the same work as N = 1 -- one 2^28-sample channel of its own -- so the N = 1,
2, 4, 8 values form one weak-scaling series (no collective in the timed
region).  Beside it, in the same line at N > 1 (at N = 1 with --share),
`configs2_share` measures configs[2]'s layout: 8 channels of 2^28 per GPU (64
over 8 GPUs), one batched step per rank (weak scaling too), and the RCCL
gather of every channel's decimated output to rank 0 (32 GiB at N = 8), timed
apart.
--channels-per-gpu C makes C channels per GPU the main series instead.

Other workloads (--workload): mixdecim (config 4, mixer -> fixed-point
decimator, fused), corr (config 5, 1024-lag correlator), fir (config 1 shape on
the GPU), up (interpolator), fifo / iq (host -> HBM ring or capture replay
feeding config 4's chain; bound by the host link).

Reported beside the GPU number:
  roofline      dominant kernel's algorithmic bytes / its HIP-event time, vs 8 TB/s
  cpu_baseline  the REFERENCE (oracle/_ref, g++ -O2) timed on this host, 1 thread
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (in) for 127-tap cplx<float> decim-4 polyphase FIR, 256 Msamp; %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TOPS = 39.32  # 256 CUs x 4 SIMD x 16 lanes x 2.4 GHz, one v_dot2 each per clock
# i8 matrix cores: v_mfma_i32_32x32x32_i8 in 32 cycles per SIMD = 1024 MACs per
# clock per SIMD (MI355X_MICROARCH.md, I8 row: 2x BF16 per clock), x 1024 SIMDs x 2.4 GHz
I8_MFMA_PEAK_MACS = 1024 * 1024 * 2.4e9
# config 5 exactly on them (scripts/tune/corr_mfma.hip): 4 limb products x 4 real
# products per complex tap = 16 i8 MACs, 1024 taps + the 3 % Toeplitz pad (66
# sixteen-sample chunks per 1024 outputs) = 16896 MACs per output
CORR_I8_MACS_PER_SAMPLE = 16896.0
SEED = 0x5EED


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # The chip's clocks settle only after ~50 back-to-back launches (measured:
    # steps 0-20 of a cold start average 0.65 ms for the headline, 0.49 ms from
    # step 50 on -- profiles/r01_warmup_ramp_*.txt), so the default warm-up
    # is 100 untimed steps before 200 timed ones (~0.15 s of GPU time).
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--workload", default="decim", choices=["decim", "mixdecim", "ci16decim", "corr", "fir", "up", "fifo", "iq"])
    p.add_argument("--samples", type=int, default=None,
                   help="input samples per channel per step (default 2^28; corr: 2^26, config 5's 64 Msamp)")
    # default (decim): one 2^28 channel per GPU at every N (configs[1]'s work
    # per GPU), plus the configs[2] per-GPU share (8 channels) beside it; see
    # channel_layout() and share_layout()
    p.add_argument("--channels-per-gpu", type=int, default=None)
    p.add_argument("--no-share", action="store_true", help="skip the configs[2] per-GPU share measurement (N > 1)")
    p.add_argument("--share", action="store_true",
                   help="measure the configs[2] per-GPU share at N = 1 too (default: N > 1 only, so the N = 1 "
                        "command's kernel trace holds the headline's launches alone)")
    p.add_argument("--fp", default="fma", choices=["fma", "strict"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=1 << 27, help="samples timed on the reference CPU path")
    p.add_argument("--no-gather", action="store_true")
    p.add_argument("--no-pcie", action="store_true", help="skip the host-vector (PCIe-inclusive) side measurement")
    p.add_argument("--dump-steps", action="store_true", help="print every timed step's kernel ms to stderr")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--dry-run", action="store_true",
                   help="start the ranks, rendezvous over gloo, print each rank's view of the world, exit "
                        "before any GPU call (tests the launcher on a CPU host)")
    p.add_argument("--no-parity", action="store_true",
                   help="skip the post-timing digest check of the decimated channels")
    p.add_argument("--digests", default=os.path.join(ROOT, "tests", "golden", "channel_digests.json"))
    return p.parse_args(argv)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int | None:
    """`bench.py --gpus N` (N > 1) run without a launcher: start N ranks of
    this script under torch.distributed.run as a CHILD process (one rank per
    GPU, rendezvous on 127.0.0.1) and return its exit code.  Called before
    torch, srcdsp_amd or the GPU is touched; the parent never execs.  Rank 0's
    JSON line reaches our stdout through the inherited file descriptors.
    Returns None when this process is itself a rank (WORLD_SIZE set by a
    launcher) or N == 1."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench: starting {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


CONFIG2_CHANNELS, CONFIG2_PER_GPU = 64, 8  # BASELINE configs[2]: 64 channels, 8 per GPU at N = 8


def layout_label(cpg: int, world: int) -> str:
    """Which BASELINE config a decim layout is: configs[1] is one 2^28
    channel on one GPU, configs[2] is 64 channels, 8 per GPU on 8 GPUs; the
    same per-GPU layouts at other N say so instead of claiming the config."""
    if cpg == 1:
        return "configs[1]" if world == 1 else f"configs[1] on each of {world} GPUs ({world} independent channels)"
    if cpg == CONFIG2_PER_GPU:
        total = cpg * world
        return "configs[2]" if total == CONFIG2_CHANNELS else \
            f"configs[2] per-GPU layout ({total} of {CONFIG2_CHANNELS} channels)"
    return "custom"


def channel_layout(args, world: int, L: int | None = None) -> dict:
    """Channel layout of the main series (decim workload): one 2^28-sample
    channel per GPU at every N unless --channels-per-gpu says otherwise, so
    the per-GPU work is the same at N = 1, 2, 4, 8 (weak scaling).  Channels
    are block-partitioned (srcdsp_amd.dist.channels_for_rank).  Other
    workloads run one buffer per rank.  The main series has no collective;
    the gather belongs to the configs[2] share (share_layout)."""
    if L is None:
        L = args.samples if args.samples is not None else (1 << 28)
        L -= L % 4
    if args.workload != "decim":
        cpg = 1
    elif args.channels_per_gpu is not None:
        cpg = args.channels_per_gpu
    else:
        cpg = 1
    total = cpg * world
    return {"channels_per_gpu": cpg, "channels_total": total, "samples_per_channel": L,
            "baseline_config": layout_label(cpg, world) if args.workload == "decim" else None}


def share_layout(args, world: int, L: int | None = None) -> dict | None:
    """configs[2]'s per-GPU share measured beside the main series: 8 channels
    of 2^28 per GPU (64 in all at N = 8), and the gather of every channel's
    decimated output to rank 0.  Measured at N > 1 (and at N = 1 with
    --share: the driver's N = 1 command then profiles the headline's launches
    alone); None when not measured (other workloads, an explicit
    --channels-per-gpu, --no-share)."""
    if args.workload != "decim" or args.channels_per_gpu is not None or getattr(args, "no_share", False):
        return None
    if world == 1 and not getattr(args, "share", False):
        return None
    if L is None:
        L = args.samples if args.samples is not None else (1 << 28)
        L -= L % 4
    total = CONFIG2_PER_GPU * world
    return {"channels_per_gpu": CONFIG2_PER_GPU, "channels_total": total, "samples_per_channel": L,
            "baseline_config": layout_label(CONFIG2_PER_GPU, world),
            "gather_bytes": total * (L // 4) * 8 if use_pg(world) else 0}


def dry_run(args) -> None:
    """One line per rank: the rank/world the launcher gave it and the world a
    gloo process group actually assembled (an all-reduce of ones).  No GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    seen = 1
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    # one write() per line: the ranks share the launcher's stdout pipe, and a
    # print() (text, then newline) from two ranks can interleave on one line
    sys.stdout.flush()
    os.write(1, (json.dumps({"dry_run": True, "rank": rank, "world": world, "world_seen": seen,
                             "gpus": args.gpus, "workload": args.workload,
                             "layout": channel_layout(args, world),
                             "share_layout": share_layout(args, world)}) + "\n").encode())
    if world != args.gpus or seen != args.gpus:
        raise SystemExit(f"bench: rank {rank} sees world {world}/{seen}, --gpus {args.gpus}")


class CudaDevice:
    """Every device call bench.py makes, in one place: torch.cuda on the GPU
    box.  HostDevice (below) stands in for it in the CPU rehearsal of main()
    (tests/test_bench_cpu.py), which drives the whole N > 1 path -- timing,
    parity digests, configs[2] share, gather, line assembly -- on gloo ranks
    with a host stand-in for the operators."""
    name = "cuda"

    def __init__(self):
        import torch
        self.torch = torch

    def set_device(self, i):
        self.torch.cuda.set_device(i)

    def device_count(self):
        return self.torch.cuda.device_count()

    def synchronize(self):
        self.torch.cuda.synchronize()

    def stream(self):
        return self.torch.cuda.current_stream()

    def event_pair(self):
        E = self.torch.cuda.Event
        return E(enable_timing=True), E(enable_timing=True)

    def empty_cache(self):
        self.torch.cuda.empty_cache()


class _HostEvent:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


class HostDevice(CudaDevice):
    """Host stand-in for CudaDevice (CPU rehearsal only: its times are host
    wall times of the stand-in operators, never a measurement)."""
    name = "cpu"

    def __init__(self):
        pass

    def set_device(self, i):
        pass

    def device_count(self):
        return 1

    def synchronize(self):
        pass

    def stream(self):
        return None

    def event_pair(self):
        return _HostEvent(), _HostEvent()

    def empty_cache(self):
        pass


DEV = None  # set by main(): CudaDevice() unless a HostDevice is passed in

# "nccl" (= RCCL over xGMI) on a multi-GPU node.  SRCDSP_BENCH_BACKEND=gloo is
# only for rehearsing the N > 1 code path with several ranks on ONE GPU (the
# collectives then move host copies); its timings are not scaling numbers.
BACKEND = os.environ.get("SRCDSP_BENCH_BACKEND", "nccl")
COLL_DEV = "cuda" if BACKEND == "nccl" else None  # device of the collectives' small tensors
# SRCDSP_BENCH_PG=1: a process group (and every collective of the N > 1 path:
# barriers, MAX of the wall times, parity SUMs, the share's gather, the
# correlator's MIN) even at WORLD_SIZE 1 -- the N > 1 path on the real backend
# on a one-GPU box, as a rehearsal; the line is the same work as N = 1
FORCE_PG = os.environ.get("SRCDSP_BENCH_PG") == "1"


def use_pg(world: int) -> bool:
    return world > 1 or FORCE_PG


def dist_setup(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if use_pg(world):
        import torch.distributed as dist
        if BACKEND == "nccl":
            DEV.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            DEV.set_device(local % DEV.device_count())
            dist.init_process_group("gloo")
    else:
        DEV.set_device(0)
    return world, rank, local


def barrier(world):
    if use_pg(world):
        import torch.distributed as dist
        dist.barrier()
    DEV.synchronize()


# ---------------------------------------------------------------- workloads
class Workload:
    """One step = one pass of the hot path over one batch of resident input."""
    name = ""
    bytes_per_sample = 0.0   # algorithmic HBM bytes per input sample
    dtype = ""

    def step(self):
        raise NotImplementedError


class DecimWorkload(Workload):
    dtype = "f32"
    bytes_per_sample = 10.0  # 8 B complex<float> read + 8 B out per 4 inputs
    read_bytes_per_sample = 8.0

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd.design import hamming_sinc
        self.c = hamming_sinc(127)
        self.L, self.C = L, channels
        self.x = torch.empty((channels, L), dtype=torch.complex64, device=DEV.name)
        for ch in range(channels):
            S.fill_synthetic(self.x[ch], "cf32", seed=SEED, channel=rank * channels + ch)
        self.y = torch.empty((channels, L // 4), dtype=torch.complex64, device=DEV.name)
        self.f = [S.FilterDnsamplingFir(self.c, 4, fp=fp) for _ in range(channels)]
        self.S = S
        self.name = "decim_cf32_m4_t127"

    def step(self):
        if self.C == 1:
            self.f[0].step(self.x[0], self.y[0])
        else:
            self.S.decim_step_batched(self.f, self.x, self.y)


class MixDecimWorkload(Workload):
    dtype = "i32"
    bytes_per_sample = 5.0  # 4 B complex<int16_t> read + 4 B out per 4 inputs
    read_bytes_per_sample = 4.0
    # algorithmic dot2 work per input sample: the decimator's 127 taps x 2
    # components per output, 1 output per 4 inputs = 63.5 int MACs = 31.75
    # v_dot2 lane-ops (the kernel issues 32: 64 tap pairs, the last with a zero
    # tap), plus the mixer's complex product = 4 MACs = 2 v_dot2
    dot2_per_sample = 33.75

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd.design import hamming_sinc, q14
        cq = q14(hamming_sinc(127))
        self.x = torch.empty((L, 2), dtype=torch.int16, device=DEV.name)
        S.fill_synthetic(self.x, "ci16", seed=SEED, channel=rank, lo=-8192, hi=8191)
        self.y = torch.empty((L // 4, 2), dtype=torch.int16, device=DEV.name)
        m = S.Mixer(4096)
        m.reset(0.1)
        d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
        self.chain = S.MixerDecimatorChain(m, d)
        self.name = "mixer4096_f0.1_to_decim_ci16_q14_m4_t127"

    def step(self):
        self.chain.step(self.x, self.y)


class CorrWorkload(Workload):
    """Config 5.  One 64 Msamp buffer; at N > 1 it is split in time (SURVEY
    8e): rank r primes its correlator with the N*S+2 samples before its share,
    scans its share, and the first detection is a MIN all-reduce over RCCL."""
    dtype = "i32"
    bytes_per_sample = 4.0

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd import dist as D
        from srcdsp_amd.design import qpsk_pattern
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.p = qpsk_pattern(1024, 500, seed=2)
        rng = np.random.default_rng(0)  # the same global buffer on every rank
        x = rng.integers(-125, 126, size=(L, 2)).astype(np.int32)
        off = (3 * L) // 4
        x[off:off + 1024] += 2 * self.p
        x = np.clip(x, -32768, 32767).astype(np.int16)
        self.s0, s1 = D.time_segment(L, self.world, rank)
        hc = min(self.s0, D.corr_halo(1024, 1))
        self.halo = torch.from_numpy(x[self.s0 - hc:self.s0]).cuda() if hc else None
        self.x = torch.from_numpy(x[self.s0:s1]).cuda()
        del x
        self.S, self.D = S, D
        self.name = "corr_1024x1"
        self.expect = off + 1023  # corrIndex = the peak sample (pattern end), reported one sample later
        self.g = S.FixedPatternCorrelator(1024, 1)
        self.g.setPattern(self.p)

    def step(self):
        # one independent 64 Msamp buffer per step: reset() (correlators.h:196)
        # clears the registers and history, then one step() scans to the hit
        self.g.reset()
        local = self.D.corr_segment_search(self.g, self.halo, self.x, self.s0)
        first = self.D.first_detection(local, self.world, device=COLL_DEV)
        found = first != self.D.NO_DETECTION
        self.last = (found, first if found else -1)


class FirWorkload(Workload):
    dtype = "f32"
    bytes_per_sample = 12.0  # 4 B float in, 8 B complex<float> out
    read_bytes_per_sample = 4.0

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd.design import hamming_sinc
        self.x = torch.randint(-2048, 2048, (L,), device=DEV.name).float()
        self.y = torch.empty(L, dtype=torch.complex64, device=DEV.name)
        self.f = S.FilterFir(hamming_sinc(31, 0.2), "float", "complex<float>", "float", "float", fp=fp)
        self.name = "fir_f32_t31"

    def step(self):
        self.f.step(self.x, self.y)


class UpWorkload(Workload):
    """FilterUpsamplingFir<ci16,ci16,ci32,int32_t,4> (a7; not a BASELINE config):
    128-tap Q14 interpolator, L = 4, input length L samples -> 4L outputs."""
    dtype = "i32"
    bytes_per_sample = 20.0  # 4 B complex<int16_t> in, 4 x 4 B out per input sample
    read_bytes_per_sample = 4.0
    # 4 outputs per input, 32 taps each, 2 components: 256 int MACs = 128 v_dot2
    # lane-ops per input sample (the kernel issues exactly these: 16 tap pairs
    # (c[2p+1], c[2p]) per phase and component)
    dot2_per_sample = 128.0

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd.design import hamming_sinc, q14
        n = L // 4  # keep the output (4n samples) the size of the other workloads' input
        self.x = torch.empty((n, 2), dtype=torch.int16, device=DEV.name)
        S.fill_synthetic(self.x, "ci16", seed=SEED, channel=rank, lo=-8192, hi=8191)
        self.y = torch.empty((4 * n, 2), dtype=torch.int16, device=DEV.name)
        self.f = S.FilterUpsamplingFir(q14(hamming_sinc(128, 0.12) * 4), 4)
        self.n = n
        self.name = "up_ci16_q14_l4_t128"

    def step(self):
        self.f.step(self.x, self.y)


class Ci16DecimWorkload(Workload):
    """SURVEY §8a row a2 on its own: FilterDnsamplingFir<ci16,ci16,ci32,int32_t,4>,
    127 Q14 taps, no mixer (config 4's decimator)."""
    dtype = "i32"
    bytes_per_sample = 5.0
    read_bytes_per_sample = 4.0
    dot2_per_sample = 31.75  # 127 taps x 2 components / 4 = 63.5 int MACs (the kernel issues 32 dot2)

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd.design import hamming_sinc, q14
        cq = q14(hamming_sinc(127))
        self.x = torch.empty((L, 2), dtype=torch.int16, device=DEV.name)
        S.fill_synthetic(self.x, "ci16", seed=SEED, channel=rank, lo=-8192, hi=8191)
        self.y = torch.empty((L // 4, 2), dtype=torch.int16, device=DEV.name)
        self.d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
        self.name = "decim_ci16_q14_m4_t127"

    def step(self):
        self.d.step(self.x, self.y)


def _mixdecim_chain(S):
    """config 4's operators: Mixer<ci16,ci16,int16_t,4096> at f = 0.1 feeding the
    127-tap Q14 FilterDnsamplingFir<ci16,ci16,ci32,int32_t,4>"""
    from srcdsp_amd.design import hamming_sinc, q14
    m = S.Mixer(4096)
    m.reset(0.1)
    d = S.FilterDnsamplingFir(q14(hamming_sinc(127)), 4, "complex<int16_t>", "complex<int16_t>",
                              "complex<int32_t>", "int32_t")
    return S.MixerDecimatorChain(m, d)


class FifoWorkload(Workload):
    """SURVEY 8f.3 (the caller side of the path): a host producer feeds the HBM
    FifoWithTimeTrack ring; the consumer reads each block back into a device
    buffer and runs config 4's mixer -> decimator chain on it.  One step =
    write() of one host block of complex<int16_t> (memcpy into one of two
    pinned buffers, H2D on the FIFO's copy stream), read() of the same block
    (ordered after the write on the device), one chain step.  Bound: the host
    link, 4 B per sample H2D."""
    dtype = "i32"
    bytes_per_sample = 4.0  # H2D bytes per sample (the ring and the chain stay in HBM)
    bound = "pcie"

    def __init__(self, S, torch, L, channels, rank, fp):
        self.B = min(L, 1 << 24)
        rng = np.random.default_rng(rank)
        self.h = rng.integers(-8192, 8192, size=(self.B, 2)).astype(np.int16)
        self.fifo = S.FifoWithTimeTrack(np.dtype(("<i2", 2)), 4 * self.B)
        self.x = torch.empty((self.B, 2), dtype=torch.int16, device=DEV.name)
        self.y = torch.empty((self.B // 4, 2), dtype=torch.int16, device=DEV.name)
        self.chain = _mixdecim_chain(S)
        self.name = f"fifo_ring{4 * self.B}_block{self.B}_ci16_to_mixdecim"
        self.n = self.B

    def step(self):
        self.fifo.write(self.h)
        te = self.fifo.state()[2]
        err, _, _ = self.fifo.read(self.x, te - self.B + 1)
        if err:
            raise RuntimeError("FIFO read failed")
        self.chain.step(self.x, self.y)


class IqLoadWorkload(Workload):
    """replay of a binary I/Q capture (dsptl_files.h format) from
    a file into device memory (fread overlapped with H2D through two pinned
    chunks), then config 4's mixer -> decimator chain on it.  The file is
    written once before timing (page cache warm).  Bound: the host link,
    4 B per sample H2D."""
    dtype = "i32"
    bytes_per_sample = 4.0
    bound = "pcie"

    def __init__(self, S, torch, L, channels, rank, fp):
        from srcdsp_amd import files
        self.files = files
        self.B = min(L, 1 << 26)
        rng = np.random.default_rng(rank)
        tmp = os.environ.get("TMPDIR", "/tmp")
        self.path = os.path.join(tmp, f"srcdsp_bench_iq_{os.getpid()}_{rank}.bin")
        files.saveBinarySamples(rng.integers(-8192, 8192, size=(self.B, 2)).astype(np.int16), self.path)
        self.y = torch.empty((self.B // 4, 2), dtype=torch.int16, device=DEV.name)
        self.chain = _mixdecim_chain(S)
        self.name = f"iq_capture{self.B}_ci16_to_mixdecim"
        self.n = self.B

    def step(self):
        x = self.files.readBinarySamples(self.path, "complex<int16_t>", device=True)
        self.chain.step(x, self.y)

    def close(self):
        try:
            os.remove(self.path)
        except OSError:
            pass


WORKLOADS = {"decim": DecimWorkload, "mixdecim": MixDecimWorkload, "ci16decim": Ci16DecimWorkload, "corr": CorrWorkload, "fir": FirWorkload,
             "up": UpWorkload, "fifo": FifoWorkload, "iq": IqLoadWorkload}
PCIE_PEAK_GBS = 63.0  # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s (spec)


# ---------------------------------------------------------------- CPU baseline
def cpu_baseline(args, flavour="strict", sample=None):
    """Time the reference itself (oracle/_ref/<flavour>: strict = g++ -O2, O0 =
    the reference makefile's own flags, no -O; 1 thread) on a bounded sample
    of the same workload; test infrastructure, never the product."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    if args.workload in ("mixdecim", "corr", "fir", "up", "fifo", "iq"):
        return cpu_baseline_other(args, pyoracle)
    if args.workload != "decim":
        return None
    d = os.path.join(ROOT, "oracle", "_ref", flavour)
    path = os.path.join(d, "libref_decim_old.so")
    if flavour != "strict" and not os.path.exists(path):
        return None
    n = min(sample or args.cpu_sample, args.samples)
    n -= n % 4
    if os.path.exists(path):
        lib = C.CDLL(path)
        lib.ref_decim_create.restype = C.c_void_p
        lib.ref_decim_create.argtypes = [C.c_int, C.c_uint, C.c_void_p, C.c_int]
        lib.ref_decim_step_timed.restype = C.c_double
        lib.ref_decim_step_timed.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
        lib.ref_decim_destroy.argtypes = [C.c_void_p]
        c = hamming_sinc(127)
        h = lib.ref_decim_create(0, 4, c.ctypes.data, 127)
        x = pyoracle.Oracle(0).gen_cf32(SEED, 0, 0, n)
        y = np.zeros(n // 4, np.complex64)
        secs = lib.ref_decim_step_timed(h, x.ctypes.data, n, y.ctypes.data)
        lib.ref_decim_destroy(h)
        kind = "reference"
        src = (f"oracle/_ref/{flavour}/libref_decim_old.so (dnsampling_filters.h built g++ "
               + ("-O2, x86-64 baseline)" if flavour == "strict" else
                  "-std=gnu++11 without -O: the reference makefile's flags, /root/reference/makefile:18)"))
    else:  # no reference build travelled: time the C restatement instead
        o = pyoracle.Oracle(0)
        x = o.gen_cf32(SEED, 0, 0, n)
        f = o.decim(0, 4, hamming_sinc(127))
        t0 = time.perf_counter()
        f.step(x)
        secs = time.perf_counter() - t0
        kind = "port"
        src = "oracle/liboracle.so (C restatement, -O2)"
    cpu = ""
    try:
        with open("/proc/cpuinfo") as fh:
            cpu = next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
    except Exception:
        pass
    return {"value": round(n / secs / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": kind,
            "sample": f"{n} samples (first {n} of channel 0 of the same synthetic workload), one step() call, "
                      f"{secs:.2f} s; {src}; host CPU: {cpu}"}


def host_cores():
    """(cores this process may use, description).  SURVEY §8d asks for "all the
    nproc cores"; on a shared GPU box nproc/os.cpu_count() report the whole
    machine while this job's share is the affinity mask, further capped by the
    box's OMP_NUM_THREADS (the per-GPU CPU share, 16 on the MI355X pool)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = total
    omp = os.environ.get("OMP_NUM_THREADS")
    n = aff
    if omp and omp.isdigit() and 0 < int(omp) < n:
        n = int(omp)
    return n, (f"{n} threads = this job's CPU share (affinity mask {aff} CPUs, OMP_NUM_THREADS={omp}); "
               f"machine nproc {total}")


def cpu_topology():
    """The CPUs of this process's affinity mask and one CPU per physical core
    among them (the lowest-numbered SMT sibling of each (package, core_id),
    from /sys/devices/system/cpu/cpu*/topology)."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    first = {}
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "physical_package_id") as f:
                pkg = int(f.read())
            with open(base + "core_id") as f:
                core = int(f.read())
        except (OSError, ValueError):
            pkg, core = 0, c
        first.setdefault((pkg, core), c)
    return cpus, sorted(first.values())


def cpu_quota():
    """The cgroup CPU bandwidth limit of this process, as a note: on a shared
    GPU box the affinity mask can list every hardware thread while the
    scheduler grants the job only a quota of CPU time (cgroup v2 cpu.max, or
    v1 cfs_quota_us / cfs_period_us); threads beyond it share that time."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
        except OSError:
            continue
        if parse is not None:
            q, per = parse(txt)[:2]
        else:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                q, per = txt, f.read().strip()
        if q in ("max", "-1"):
            return f"no cgroup CPU quota ({path}: {txt})"
        return f"cgroup CPU quota {int(q) / int(per):.1f} CPUs ({path}: {txt})"
    return "cgroup CPU quota unknown"


def _ref_decim_lib():
    path = os.path.join(ROOT, "oracle", "_ref", "strict", "libref_decim_old.so")
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    lib.ref_decim_create.restype = C.c_void_p
    lib.ref_decim_create.argtypes = [C.c_int, C.c_uint, C.c_void_p, C.c_int]
    lib.ref_decim_step_timed.restype = C.c_double
    lib.ref_decim_step_timed.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
    lib.ref_decim_destroy.argtypes = [C.c_void_p]
    return lib


def _ref_threads(lib, pins, n, reps):
    """len(pins) threads, thread i pinned to CPU pins[i] (None: unpinned),
    each owning a reference FilterDnsamplingFir<cf32,...,4> (oracle/_ref/strict)
    and channel i of the synthetic workload (n samples, generated by the thread
    itself), stepping it `reps` times (the stream continues over the same
    block).  Returns (samples/s over all threads, wall seconds): all threads'
    samples / the time from the common start to the last thread's end.  ctypes
    drops the GIL for the calls."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(127)
    o = pyoracle.Oracle(0)
    T = len(pins)
    start = threading.Barrier(T + 1)
    ends = [0.0] * T
    err = []

    def run(i):
        try:
            if pins[i] is not None:
                os.sched_setaffinity(0, {pins[i]})  # this thread only (Linux: pid 0 = the calling thread)
            x = o.gen_cf32(SEED, i, 0, n)
            y = np.zeros(n // 4, np.complex64)
            h = lib.ref_decim_create(0, 4, c.ctypes.data, 127)
        except Exception as e:  # keep the barrier count right
            err.append(e)
            start.wait()
            return
        start.wait()
        for _ in range(reps):
            lib.ref_decim_step_timed(h, x.ctypes.data, n, y.ctypes.data)
        ends[i] = time.perf_counter()
        lib.ref_decim_destroy(h)

    th = [threading.Thread(target=run, args=(i,)) for i in range(T)]
    for t in th:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    if err:
        raise err[0]
    wall = max(ends) - t0
    return T * n * reps / wall, wall


def cpu_baseline_allcores(args, threads=None):
    """the reference on ALL the host's cores, one independent
    channel per thread (config 3's layout): every hardware thread of the
    affinity mask (= nproc on the GPU box), and one thread per physical core;
    beside them the job's CPU share (host_cores(): 16 threads on the MI355X
    pool).  Each thread is pinned to its CPU and steps its own reference
    object (oracle/_ref/strict, g++ -O2) over 2^22 samples of its channel 4
    times (2^24 samples per thread, bounded host memory: 128 MiB of samples per
    thread).  `threads` (tests) replaces the three runs by one unpinned run of
    that many threads."""
    if args.workload != "decim":
        return None
    lib = _ref_decim_lib()
    if lib is None:
        return None
    n = min(1 << 22, args.samples)
    n -= n % 4
    reps = 4
    model = _cpu_model()

    def fig(pins, what):
        rate, wall = _ref_threads(lib, pins, n, reps)
        return {"value": round(rate / 1e6, 3), "unit": "Msamples/s", "cores": len(pins), "kind": "reference",
                "sample": f"{len(pins)} threads ({what}) x {reps} x {n} samples (channel i of the synthetic "
                          f"workload on thread i, one FilterDnsamplingFir per thread), {wall:.2f} s wall; "
                          f"oracle/_ref/strict/libref_decim_old.so; host CPU: {model}"}

    if threads is not None:
        return fig([None] * threads, "caller-set, unpinned")
    cpus, phys = cpu_topology()
    share, share_note = host_cores()
    out = fig(cpus, f"every hardware thread of the affinity mask, machine nproc {os.cpu_count()}")
    out["physical_cores"] = fig(phys, "one per physical core")
    out["job_share"] = fig(cpus[:share], share_note)
    out["cpu_quota"] = cpu_quota()
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            return next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
    except Exception:
        return ""


def cpu_baseline_other(args, pyoracle):
    """Reference (oracle/_ref/strict, g++ -O2, 1 thread) for configs 4 and 5,
    timed around the harness calls (includes its std::vector copies, a few %)."""
    from srcdsp_amd.design import hamming_sinc, q14, qpsk_pattern
    if not pyoracle.reference_available("strict"):
        return None
    ref = pyoracle.Reference("strict")
    o = pyoracle.Oracle(0)
    if args.workload == "ci16decim":
        n = min(1 << 25, args.samples)
        n -= n % 4
        x = o.gen_ci16(SEED, 0, 0, n, -8192, 8191)
        d = ref.decim(1, 4, q14(hamming_sinc(127)))
        t0 = time.perf_counter()
        d.step(x)
        secs = time.perf_counter() - t0
        what = "FilterDnsamplingFir<ci16,ci16,ci32,int32_t,4>::step, 127 Q14 taps"
    elif args.workload in ("mixdecim", "fifo", "iq"):
        n = min(1 << 25, args.samples)
        n -= n % 4
        x = o.gen_ci16(SEED, 0, 0, n, -8192, 8191)
        m = ref.mixer(4096)
        m.reset(0.1)
        d = ref.decim(1, 4, q14(hamming_sinc(127)))
        t0 = time.perf_counter()
        d.step(m.step(x))
        secs = time.perf_counter() - t0
        what = "Mixer<ci16,ci16,int16_t,4096>::step then FilterDnsamplingFir<ci16,ci16,ci32,int32_t,4>::step"
        if args.workload != "mixdecim":
            what += (" (the chain this workload feeds; the reference's FIFO/file hop is a memcpy beside it, "
                     "not timed)")
    elif args.workload == "fir":
        n = min(1 << 25, args.samples)
        x = np.random.default_rng(0).integers(-2048, 2048, n).astype(np.float32)
        f = ref.fir(1, hamming_sinc(31, 0.2))
        t0 = time.perf_counter()
        f.step(x)
        secs = time.perf_counter() - t0
        what = "FilterFir<float,complex<float>,float,float>::step, 31 taps (config 1's operator)"
    elif args.workload == "up":
        n = min(1 << 21, args.samples // 4)
        x = o.gen_ci16(SEED, 0, 0, n, -8192, 8191)
        u = ref.up(0, 4, q14(hamming_sinc(128, 0.12) * 4))
        t0 = time.perf_counter()
        u.step(x)
        secs = time.perf_counter() - t0
        what = "FilterUpsamplingFir<ci16,ci16,ci32,int32_t,4>::step, 128 taps (input samples/s)"
    else:
        n = min(1 << 22, args.samples)
        p = qpsk_pattern(1024, 500, seed=2)
        rng = np.random.default_rng(0)
        x = np.clip(rng.integers(-125, 126, size=(n, 2)), -32768, 32767).astype(np.int16)
        c = ref.corr(1024, 1)
        c.set_pattern(p)
        t0 = time.perf_counter()
        c.step(x)
        secs = time.perf_counter() - t0
        what = "FixedPatternCorrelator<int16_t,int32_t,1024,1>::step (noise, no detection: full scan)"
    return {"value": round(n / secs / 1e6, 4), "unit": "Msamples/s", "cores": 1, "kind": "reference",
            "sample": f"{n} samples of the same workload, {secs:.2f} s; {what}; oracle/_ref/strict (g++ -O2); "
                      f"host CPU: {_cpu_model()}"}


def host_leg(fn, *a, **kw):
    """A host-side leg of the line (CPU baselines): its failure on an unusual
    host (no reference build, a CPU the affinity call refuses) is reported in
    the line instead of losing the line after the GPU measurement."""
    try:
        return fn(*a, **kw)
    except Exception as e:  # noqa: BLE001
        print(f"bench: {fn.__name__} failed: {e!r}", file=sys.stderr, flush=True)
        return {"error": f"{type(e).__name__}: {e}"}


def pcie_inclusive(S):
    """The reference-style host std::vector step() (srcdsp_decim_step_host):
    host input staged through pinned memory, H2D, the same kernel, D2H.  A side
    figure, never `value`."""
    from srcdsp_amd.design import hamming_sinc
    n = 1 << 26
    x = np.random.default_rng(0).integers(-2048, 2048, size=(n, 2)).astype(np.float32).view(np.complex64).reshape(n)
    y = np.empty(n // 4, np.complex64)
    f = S.FilterDnsamplingFir(hamming_sinc(127), 4)
    f.step(x, y)  # warm (pinned staging allocation)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        f.step(x, y)
    secs = (time.perf_counter() - t0) / reps
    return {"value": round(n / secs / 1e6, 1), "unit": "Msamples/s",
            "sample": f"{n} samples per host-vector step(), mean of {reps}: memcpy to pinned, H2D, kernel, "
                      "D2H, memcpy out (10 B/sample over PCIe)"}


def pmc_traffic(args, work_name, per_launch_samples):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (see
    profiles/README.md for how it is collected and corrected), if it was
    measured on this launch size AND on the current kernel sources (its
    `kernel_sources_sha` against srcdsp_amd.build.source_digest(workload):
    the translation unit of the kernel and its headers).  Returns
    (bytes or None, note)."""
    from srcdsp_amd.build import source_digest
    try:
        with open(args.traffic_json) as f:
            t = json.load(f)
    except Exception:
        return None, "no PMC summary"
    ch = args.channels_per_gpu if args.workload == "decim" else 1
    e = t.get(work_name + (f"x{ch}" if ch > 1 else ""))  # a batched launch has its own entry
    if not e or int(e.get("samples_per_launch", -1)) != per_launch_samples:
        return None, "no PMC summary for this workload size"
    if e.get("kernel_sources_sha") != source_digest(args.workload):
        print(f"bench: WARNING {args.traffic_json} entry {work_name} predates the current kernel sources; "
              "traffic not reported (re-run scripts/pmc_traffic.py)", file=sys.stderr, flush=True)
        return None, "stale: PMC summary predates the current kernel sources"
    return e.get("hbm_bytes_per_launch"), "rocprofv3 PMC, " + e.get("correction", "")


# ---------------------------------------------------------------- parity
def _load_digests(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def channel_parity(work, args, rank, table) -> dict:
    """Cross-rank parity of the decim workload (outputs on 1/2/4/8
    GPUs bit-identical to 1), checked after the timed region: every filter of
    the rank is reset() (dnsampling_filters.h:56-60) and stepped once over its
    resident channel(s), and the sha256 of each channel's output is compared
    with tests/golden/channel_digests.json (made offline from the oracle and
    the reference build by tests/golden/gen_channel_digests.py, for channel
    ids rank * C + c).  Returns this rank's counts; reduce_parity() sums them
    over ranks.  The outputs stay in work.y for the gather."""
    import concurrent.futures as cf
    import hashlib
    C_ = work.C
    first = rank * C_
    want = ((table or {}).get("digests", {}).get(args.fp, {}).get(str(work.L), {}))
    for f in work.f:
        f.reset()
    work.step()
    DEV.synchronize()

    def one(k):
        return hashlib.sha256(work.y[k].cpu().numpy().tobytes()).hexdigest()

    with cf.ThreadPoolExecutor(min(8, C_)) as ex:
        got = list(ex.map(one, range(C_)))
    checked = mism = missing = 0
    bad = []
    for k, h in enumerate(got):
        w = want.get(str(first + k))
        if w is None:
            missing += 1
        elif w == h:
            checked += 1
        else:
            checked += 1
            mism += 1
            bad.append(first + k)
    return {"channels_checked": checked, "mismatches": mism, "missing": missing, "bad_channels": bad}


def gathered_parity(bufs, args, L, table) -> dict:
    """Rank 0: the same digests over what the gather delivered (rank r's block
    holds channels 8r..8r+7), so the collective's bytes are checked too."""
    import concurrent.futures as cf
    import hashlib
    want = ((table or {}).get("digests", {}).get(args.fp, {}).get(str(L), {}))
    jobs = [(r, k) for r in range(len(bufs)) for k in range(bufs[r].shape[0])]

    def one(rk):
        r, k = rk
        return rk, hashlib.sha256(bufs[r][k].cpu().numpy().tobytes()).hexdigest()

    checked = mism = missing = 0
    per = bufs[0].shape[0]
    with cf.ThreadPoolExecutor(8) as ex:
        for (r, k), h in ex.map(one, jobs):
            w = want.get(str(r * per + k))
            if w is None:
                missing += 1
            else:
                checked += 1
                mism += int(w != h)
    return {"channels_checked": checked, "mismatches": mism, "missing": missing}


def reduce_parity(p: dict, world: int) -> dict:
    """SUM of the per-rank counts over ranks (bad channel ids: rank 0's view
    plus the total count)."""
    if use_pg(world):
        import torch
        import torch.distributed as dist
        t = torch.tensor([p["channels_checked"], p["mismatches"], p["missing"]], dtype=torch.int64,
                         device=COLL_DEV)
        dist.all_reduce(t)
        p = dict(p, channels_checked=int(t[0]), mismatches=int(t[1]), missing=int(t[2]))
    return p


# ---------------------------------------------------------------- timing
def timed_steps(work, args, world, torch):
    """W untimed warm-up steps, then K timed steps bracketed by barrier +
    synchronize on both sides.  Returns (max-over-ranks wall seconds, the HIP
    event duration of every timed step in ms, on the launch stream)."""
    from srcdsp_amd.dist import max_over_ranks
    stream = DEV.stream()
    for _ in range(args.warmup):
        work.step()
    barrier(world)
    ev = [DEV.event_pair() for _ in range(args.steps)]
    barrier(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        work.step()
        ev[i][1].record(stream)
    barrier(world)
    t1 = time.perf_counter()
    wall = max_over_ranks(t1 - t0, world, device=COLL_DEV)
    return wall, [a.elapsed_time(b) for a, b in ev]


def measure_share(S, torch, args, world, rank, L, slay, table=None) -> dict:
    """configs[2]'s per-GPU share beside the main series: 8 channels of 2^28
    per GPU, one batched step per rank, same warm-up/steps protocol (it runs
    right after the main series, on a warm chip); then the RCCL gather of every
    rank's decimated channels to rank 0, timed apart (never part of a value)."""
    from srcdsp_amd.dist import gather_to_root
    work = DecimWorkload(S, torch, L, slay["channels_per_gpu"], rank, args.fp)
    wall, kern_ms = timed_steps(work, args, world, torch)
    kern_avg_ms = float(np.mean(kern_ms))
    per_launch = L * slay["channels_per_gpu"]
    achieved = work.bytes_per_sample * per_launch / (kern_avg_ms * 1e-3) / 1e9
    out = {"baseline_config": slay["baseline_config"], "channels_per_gpu": slay["channels_per_gpu"],
           "channels_total": slay["channels_total"], "samples_per_channel": L,
           "value": round(per_launch * world * args.steps / wall / 1e6, 2), "unit": "Msamples/s",
           "ms_per_step": round(wall / args.steps * 1e3, 4), "scaling": "weak",
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "per_gpu": True,
                        "channels_per_launch": slay["channels_per_gpu"], "kernel_ms": round(kern_avg_ms, 4),
                        "algorithmic_bytes_per_launch": int(work.bytes_per_sample * per_launch)},
           "timed": "after the main series (warm chip); batched step over the rank's 8 channels"}
    if not args.no_parity:
        # after the timed steps: a fresh step per channel, digests vs the table
        out["parity"] = reduce_parity(channel_parity(work, args, rank, table), world)
    if use_pg(world) and not args.no_gather:
        barrier(world)
        g0 = time.perf_counter()
        bufs = gather_to_root(work.y if COLL_DEV else work.y.cpu(), world, rank)
        barrier(world)
        gather_ms = (time.perf_counter() - g0) * 1e3
        nbytes = int(world * work.y.numel() * work.y.element_size())
        assert nbytes == slay["gather_bytes"]
        out.update(gather_ms=round(gather_ms, 3), gather_bytes=nbytes,
                   gather_gbs=round(nbytes / (gather_ms * 1e-3) / 1e9, 1))
        if rank == 0 and not args.no_parity:
            out["gather_parity"] = gathered_parity(bufs, args, L, table)
        del bufs
    del work
    DEV.empty_cache()
    return out


# ---------------------------------------------------------------- main
def main(argv=None, S=None, dev=None):
    """argv: the command line (default sys.argv); S: the operator package
    (default srcdsp_amd, the HIP library); dev: CudaDevice() by default.  The
    CPU rehearsal passes a host stand-in for S and HostDevice()."""
    global DEV
    args = parse(argv)
    rc = spawn_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.dry_run:
        dry_run(args)
        return
    import torch
    DEV = dev if dev is not None else CudaDevice()
    world, rank, local = dist_setup(args)
    reported = world
    if use_pg(world):
        import torch.distributed as dist
        reported = dist.get_world_size()  # what the process group (RCCL) actually assembled
    if world != args.gpus or reported != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s) "
                         f"(process group: {reported})")
    if S is None:
        import srcdsp_amd as S
    S.lib()  # loud failure if the HIP library is missing
    if args.samples is None:
        args.samples = (1 << 26) if args.workload == "corr" else (1 << 28)
    L = args.samples - args.samples % 4
    lay = channel_layout(args, world, L)
    slay = share_layout(args, world, L)  # before channels_per_gpu is filled in
    args.channels_per_gpu = lay["channels_per_gpu"]
    work = WORKLOADS[args.workload](S, torch, L, args.channels_per_gpu, rank, args.fp)
    work_name, work_dtype = work.name, work.dtype
    wall, kern_ms = timed_steps(work, args, world, torch)
    kern_avg_ms = float(np.mean(kern_ms))
    table = parity = None
    if args.workload == "decim" and not args.no_parity:  # outside the timed region
        table = _load_digests(args.digests)
        parity = reduce_parity(channel_parity(work, args, rank, table), world)
    if args.dump_steps and rank == 0:
        print("step_ms " + " ".join(f"{v:.4f}" for v in kern_ms), file=sys.stderr, flush=True)

    units_per_rank = L * (args.channels_per_gpu if args.workload == "decim" else 1) * args.steps
    if args.workload in ("up", "fifo", "iq"):
        units_per_rank = work.n * args.steps
    total_samples = units_per_rank * world
    if args.workload == "corr":
        # the reference's step() stops at the first detection (correlators.h:296
        # `break`): the samples it processes are those up to and including the
        # one after the peak, not the whole buffer
        found, idx = work.last
        total_samples = ((idx + 2) if found else L) * args.steps
    value = total_samples / wall / 1e6
    ms_per_step = wall / args.steps * 1e3

    per_launch_samples = L * args.channels_per_gpu if args.workload == "decim" else L
    if args.workload in ("up", "fifo", "iq"):
        per_launch_samples = work.n
    achieved = work.bytes_per_sample * per_launch_samples / (kern_avg_ms * 1e-3) / 1e9
    # SURVEY 8d / north_star: the input-read stream alone against the HBM peak
    # ("HBM-read roofline"), beside `roofline` (which counts reads + writes)
    rb = getattr(work, "read_bytes_per_sample", None)
    hbm_read = None
    if rb and getattr(work, "bound", "hbm") == "hbm":
        rd = rb * per_launch_samples / (kern_avg_ms * 1e-3) / 1e9
        hbm_read = {"achieved": round(rd, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(rd / HBM_PEAK_GBS, 4),
                    "read_bytes_per_launch": int(rb * per_launch_samples), "kernel_ms": round(kern_avg_ms, 4)}
    traffic, traffic_note = pmc_traffic(args, work.name, per_launch_samples)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_note,
            "kernel": work.name, "kernel_ms": round(kern_avg_ms, 4),
            "algorithmic_bytes_per_launch": int(work.bytes_per_sample * per_launch_samples)}
    if getattr(work, "bound", "hbm") == "pcie":
        # the host link carries the samples; the step time covers the host
        # staging memcpy, the H2D copy, the ring read and the chain kernel
        gbs = work.bytes_per_sample * per_launch_samples / (kern_avg_ms * 1e-3) / 1e9
        roof = {"bound": "pcie", "achieved": round(gbs, 2), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / PCIE_PEAK_GBS, 4), "traffic": None, "kernel": work.name,
                "kernel_ms": round(kern_avg_ms, 4), "note": "whole step on the consumer stream (host -> HBM -> chain)"}
    dps = getattr(work, "dot2_per_sample", None)
    if dps:
        # integer kernels on v_dot2: the VALU roofline beside the HBM one; the
        # binding resource (higher fraction) is `roofline`, the other rides along
        tops = dps * per_launch_samples / (kern_avg_ms * 1e-3) / 1e12
        valu = {"bound": "valu", "achieved": round(tops, 2), "peak": VALU_PEAK_TOPS, "unit": "T v_dot2 lane-ops/s",
                "frac": round(tops / VALU_PEAK_TOPS, 4), "traffic": None, "kernel": work.name,
                "kernel_ms": round(kern_avg_ms, 4), "dot2_per_input_sample": dps}
        if valu["frac"] > roof["frac"]:
            # HBM bytes per launch are the kernel's traffic whichever bound binds
            valu.update(traffic=roof["traffic"], traffic_source=roof.get("traffic_source"))
            roof, other = valu, roof
        else:
            other = valu
        roof = dict(roof, other_bound=other)
    if args.workload == "mixdecim":
        # the tap loop on the i8 matrix cores behind this C ABI (tuning build,
        # never this line's library; north_star keeps the path on vector MACs)
        roof["mfma_i8_build"] = "scripts/tune/mixdecim_mfma_step.h; profiles/tuning/r06k_mixlib_bench.json"
    if args.workload == "corr":
        # VALU-bound: 1024 complex taps = 4096 int MACs =
        # 2048 v_dot2 lane-ops per scanned sample; the reference scans up to and
        # including the detected sample.  Peak: 256 CUs x 64 lanes x 2.4 GHz.
        found, idx = work.last
        scanned = (idx + 2) if found else L  # single-buffer reference scan length
        dot2_tops = 2048.0 * scanned / world / (kern_avg_ms * 1e-3) / 1e12  # per GPU
        roof = {"bound": "valu", "achieved": round(dot2_tops, 2), "peak": VALU_PEAK_TOPS,
                "unit": "T v_dot2 lane-ops/s", "frac": round(dot2_tops / VALU_PEAK_TOPS, 4),
                # HBM bytes per launch (PMC), as for the other VALU-bound lines
                "traffic": traffic, "traffic_source": traffic_note,
                "kernel": work.name, "kernel_ms": round(kern_avg_ms, 4), "scanned_samples": int(scanned),
                "hbm_gbs_for_reference": round(achieved, 1)}
        # the chip-level bound of the same exact integer arithmetic (VERDICT r5
        # item 3): on the i8 matrix cores through int8 limbs.  Measured by the
        # tuning probe (bit-exact on every sample of this buffer),
        # not shipped: north_star keeps this path on vector MACs.
        rate = scanned / world / (kern_avg_ms * 1e-3)
        i8 = I8_MFMA_PEAK_MACS / CORR_I8_MACS_PER_SAMPLE
        roof["other_bound"] = {"bound": "mfma_i8", "achieved": round(rate / 1e9, 2), "peak": round(i8 / 1e9, 1),
                               "unit": "Gsamples/s", "frac": round(rate / i8, 4),
                               "formulation": "int8 limbs of the int16 samples and of the pattern, Toeplitz "
                                              "32x32x32 tiles, 16896 i8 MACs per output (exact mod 2^32)",
                               "probe": "scripts/tune/corr_mfma.py; profiles/tuning/r06_corr_mfma.json",
                               # the same kernel behind this C ABI (tuning build, never this line's library)
                               "c_abi_build": "scripts/tune/corr_mfma_scan.h; profiles/tuning/r06g_corrlib_bench.json"}

    share = None
    if slay is not None:  # beside the main workload's buffers (2.5 GiB): HBM holds both
        share = measure_share(S, torch, args, world, rank, L, slay, table)

    if rank == 0:
        cfg = {"workload": work_name, "samples_per_channel": L, "channels_per_gpu": args.channels_per_gpu,
               "channels_total": lay["channels_total"],
               "baseline_config": lay["baseline_config"],
               "taps": {"decim": 127, "mixdecim": 127, "ci16decim": 127, "fir": 31, "up": 128}.get(args.workload),
               "decimation": {"decim": 4, "mixdecim": 4, "ci16decim": 4}.get(args.workload), "interpolation": 4 if args.workload == "up" else None,
               "fp_contract": args.fp,
               "parallelism": (f"one buffer split in time over {world} GPU(s), first detection by MIN all-reduce"
                               if args.workload == "corr" else f"channels sharded over {world} GPU(s)"),
               "timed": "device-resident input, one step() per step; PCIe excluded"}
        if getattr(work, "bound", "hbm") == "pcie":
            cfg.update({"samples_per_channel": work.n, "taps": 127, "decimation": 4,
                        "timed": ("host block -> pinned staging -> H2D -> HBM (FIFO ring or capture) -> "
                                  "mixer->decimator chain, one block per step; PCIe included")})
        line = {"metric": METRIC if args.workload == "decim" else f"Msamples/sec (in), {work_name}",
                "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
                "scaling": "strong" if args.workload == "corr" and world > 1 else "weak",
                "vs_baseline": None, "dtype": work_dtype,
                "data": "synthetic (counter-based splitmix64 integer samples, SURVEY §8d)", "config": cfg,
                "roofline": roof, "hbm_read": hbm_read, "world_size_reported": reported,
                "backend": BACKEND if use_pg(world) else None}
        if args.workload == "decim":
            # `roofline` is rank 0's own launch(es): per GPU, the same work at every N
            roof["per_gpu"] = True
            roof["channels_per_launch"] = args.channels_per_gpu
        if parity is not None:
            line["parity"] = dict(parity, digest_table=os.path.relpath(args.digests, ROOT), fp_contract=args.fp,
                                  checked=("after the timed region: every rank resets its filters, steps its "
                                           "resident channel(s) once, and compares sha256 of each channel's output "
                                           "with the oracle/reference digest of that channel id; counts summed "
                                           "over ranks"))
        if share is not None:
            line["configs2_share"] = share
        if args.workload == "corr":
            line["detection"] = list(work.last)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = host_leg(cpu_baseline, args)
            if args.workload == "decim":
                line["cpu_baseline_allcores"] = host_leg(cpu_baseline_allcores, args)
                # the reference-equivalent -O0 build, for context
                line["cpu_baseline_O0"] = host_leg(cpu_baseline, args, "O0", sample=1 << 24)
        if args.workload == "decim" and world == 1 and not args.no_pcie:
            line["pcie_inclusive"] = pcie_inclusive(S)
        print(json.dumps(line), flush=True)
    if hasattr(work, "close"):
        work.close()
    if use_pg(world):
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
