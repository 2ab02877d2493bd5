"""Benchmark: ResNet-18-depsep 225x225 training step (BASELINE config 3; config 4 with --gpus N).

One step = forward (loss) + backward + SGD-momentum update of the whole network on one
synthetic batch of 256 images per GPU (fp32), inputs resident in HBM before timing.
Multi-GPU: one process per GPU (torchrun), data parallel over RCCL, per-rank batch fixed
(weak scaling); gradients are averaged with bucketed all-reduces overlapped with backward.

Prints ONE JSON line (rank 0).  Besides the driver's contract fields it carries
  roofline      -- the dominant kernel (largest share of the step, measured with HIP events
                   around every call of that C-ABI entry point during a second run of the K
                   timed steps; `value` comes from the first, uninstrumented run):
                   algorithmic work per call / average call duration vs the MI355X peak;
  cpu_baseline  -- the reference's CPU path restated (oracle/cpu_path.py: C/OpenMP versions
                   of its Cython kernels + numpy BLAS), timed on this host at N=1 on a small
                   sample of the same workload;
  breakdown     -- per entry point: ms per step and roofline fraction (one instrumented step,
                   run single-stream; the timed steps run the weight gradients on a side
                   stream, so the breakdown sums to more than ms_per_step).
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec training step, ResNet-18-depsep 225x225 bs=256, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 20 (config 2: 50)")
    ap.add_argument("--warmup", type=int, default=None, help="default 10 (config 2: 20)")
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--bn", choices=["local", "sync"], default="local")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=32, help="images per CPU-baseline step (0 = skip)")
    ap.add_argument("--cpu-steps", type=int, default=10, help="timed CPU-baseline steps (median reported)")
    ap.add_argument("--cpu-warmup", type=int, default=2, help="untimed CPU-baseline steps")
    ap.add_argument("--config", type=int, choices=[1, 2, 3, 5], default=3,
                    help="BASELINE config: 3 (default; 4 with --gpus N) = ResNet-18-depsep training step; "
                         "1 = MNISTNet bs=64 training step; 2 = single 3x3 ConvLayer fwd+dgrad+wgrad; "
                         "5 = bf16 depthwise-separable stack (secondary lines, not the headline metric)")
    ap.add_argument("--pmc", default=None,
                    help="per-kernel HBM traffic from rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same command "
                         "(scripts/pmc_summary.py output; default: the newest summary of this config in "
                         "profiles/pmc_index.json)")
    ap.add_argument("--knob", action="append", default=[], metavar="KIND=V",
                    help="A/B runs: dk_debug_set_gemm_config(KIND, V) before the run (include/dorknet_hip.h)")
    a = ap.parse_args()
    # enough warmup for the clocks to settle (the first timed steps after 3 warmups ran up to 5 %
    # slow, profiles/r03s_cfg2_rows.txt round 1), and more steps for config 2's 1.6 ms pass
    if a.steps is None:
        a.steps = 50 if a.config == 2 else 20
    if a.warmup is None:
        a.warmup = 20 if a.config == 2 else 10
    return a


class Instrument:
    """Wraps C-ABI entry points so every call is bracketed by HIP events on the current
    stream (the stream the kernels are launched on)."""

    def __init__(self, names, reserve=0):
        """reserve: event pairs created up front (the timed region's calls), so that the wrapper
        only records them -- creating two events per call costs host time in the timed loop."""
        import torch
        from dorknet_amd._hip import lib
        self.lib = lib
        self.names = list(names)
        self.calls = {n: [] for n in self.names}
        self.orig = {}
        self.pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                     for _ in range(reserve)]

    def __enter__(self):
        import torch
        for n in self.names:
            orig = getattr(self.lib, n)
            self.orig[n] = orig
            calls = self.calls[n]

            def wrapped(*args, _orig=orig, _calls=calls, _pool=self.pool):
                if _pool:
                    e0, e1 = _pool.pop()
                else:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                r = _orig(*args)
                e1.record()
                _calls.append((e0, e1, args))
                return r
            setattr(self.lib, n, wrapped)
        return self

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(self.lib, n, f)

    def summary(self):
        import torch
        from dorknet_amd import perfmodel
        torch.cuda.synchronize()
        out = {}
        for n, calls in self.calls.items():
            if not calls:
                continue
            ms = [a.elapsed_time(b) for a, b, _ in calls]
            fl, by = 0, 0
            bound = 0.0
            shapes = {}  # (flops, bytes) of a call -> [calls, ms]: the entry's distinct shapes
            for (_, _, args), t in zip(calls, ms):
                f, b = perfmodel.work(n, args)
                fl += f
                by += b
                bound += perfmodel.bound_time_s(f, b, n)
                sh = shapes.setdefault((f, b), [0, 0.0])
                sh[0] += 1
                sh[1] += t
            out[n] = dict(calls=len(calls), ms=sum(ms), flops=fl, bytes=by, bound_ms=1e3 * bound, shapes=shapes)
        return out


class single_stream:
    """Everything on the launch stream for the per-entry attribution step: weight gradients not
    on the side stream (DORKNET_ASYNC_WGRAD=0) and skip projections not on the branch stream
    (DORKNET_BRANCH_STREAM=0).  Otherwise an entry's events would also time the other streams'
    kernels running beside it (the skip projections' entries read 0.15 of their
    bound while they overlapped the chain)."""
    KEYS = ("DORKNET_ASYNC_WGRAD", "DORKNET_BRANCH_STREAM")

    def __enter__(self):
        self.prev = {k: os.environ.get(k) for k in self.KEYS}
        for k in self.KEYS:
            os.environ[k] = "0"
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return False


def shape_bounds(name, s):
    """Each distinct call shape of an entry with its own bound (HBM or MFMA) and its fraction of
    that bound, largest time first."""
    from dorknet_amd import perfmodel
    rows = []
    for (f, b), (n, ms) in sorted(s.get("shapes", {}).items(), key=lambda kv: -kv[1][1]):
        t = ms / 1e3 / n
        mf = perfmodel.is_mfma_bound(f, b, name)
        rows.append({"calls": n, "avg_call_us": round(1e6 * t, 2), "flops": int(f), "bytes": int(b),
                     "bound": "mfma" if mf else "hbm",
                     "frac": round(perfmodel.bound_time_s(f, b, name) / t, 4)})
    return rows


def roofline_entry(name, s, steps):
    from dorknet_amd import perfmodel
    t = s["ms"] / 1e3 / s["calls"]
    flops = s["flops"] / s["calls"]
    nbytes = s["bytes"] / s["calls"]
    mfma = perfmodel.is_mfma_bound(flops, nbytes, name)
    if mfma:
        achieved, peak, unit = flops / t / 1e12, perfmodel.peak_tflops(name), "TFLOP/s"
    else:
        achieved, peak, unit = nbytes / t / 1e9, perfmodel.PEAK_HBM_GBS, "GB/s"
    return {"kernel": name, "bound": "mfma" if mfma else "hbm", "achieved": round(achieved, 2), "peak": peak,
            "unit": unit, "frac": round(achieved / peak, 4), "traffic": None,
            "calls_per_step": s["calls"] // max(steps, 1), "avg_call_us": round(1e6 * t, 2),
            "algorithmic_per_call": {"flops": int(flops), "bytes": int(nbytes)},
            # the averaged label above hides shapes with different bounds: each shape on its own
            "by_shape": shape_bounds(name, s)}


# The kernel each single-kernel entry point launches (for the PMC traffic lookup).
ENTRY_KERNEL = {
    "dk_bn_bwd_apply_f32": "dk::bn_bwd_apply_kernel",
    "dk_bn_apply_f32": "dk::bn_apply_kernel",
    "dk_add_f32": "dk::add_kernel",
    "dk_bn_add_f32": "dk::bn_add_kernel",
    "dk_relu_bwd_f32": "dk::relu_bwd_kernel",
    "dk_relu_bwd_bn_partial_f64": "dk::bn_bwd_partial_kernel",
    # (prefix, regex): the GEMM instantiations whose A operand is the K-contiguous matrix
    # loader applying a BN backward (dgrad); the stem's weight gradient applies one on its
    # row-contiguous loader (LdMatICT) and is a different entry point
    # (and the deep kernels, pw_deep.hip, in their BatchNorm form: PLAIN = false, the last
    # template argument; the plain form is the skip projections' dk_pwconv_dgrad_f32)
    "dk_pwconv_dgrad_bnbwd_f32": [("dk::igemm_f32", r"dk::LdMatKCT<[^>]*>, dk::MatBwdDesc"),
                                  ("dk::pwd::dgrad_kernel", r", false>$"), ("dk::pwd::dgrad16_kernel", r", false>$")],
    # the pointwise forward with output statistics: the tiled engine's instantiations (1x1 image
    # view, statistics epilogue), the streaming K = C = 64 kernel and the deep kernels with
    # statistics (STATS = true; the strided skip projections are dk_pwconv_fwd_f32)
    "dk_pwconv_fwd_ex_f32": [("dk::igemm_f32", r"Img(Bn)?DescE<float, true>.*EpStoreStatsT<float>"),
                             ("dk::pws::fwd_kernel", ""), ("dk::pwd::fwd_kernel", r"^dk::pwd::fwd_kernel<\d+, \w+, true")],
    # config 5 (bf16 storage): the BN-backward-on-load pointwise dgrad (streaming K = C = 64 and deep
    # kernels, the tiled engine elsewhere), the fused depthwise backward and the depthwise forward
    "dk_pwconv_dgrad_bnbwd_bf16": [("dk::pwsh::dgrad_bnbwd_kernel", ""), ("dk::pwd16::dgrad_kernel", ""),
                                   ("dk::igemm_f32", r"dk::LdMatKCT<[^>]*>, dk::MatBwdDescE<unsigned short>")],
    "dk_pwconv_fwd_ex_bf16": [("dk::pwsh::fwd_kernel", ""), ("dk::pwd16::fwd_kernel", "")],
    "dk_dwconv_bwd_bnbwd_bf16": ("dk::dw_bwd_fused_kernel", r"unsigned short"),
    "dk_dwconv_fwd_ex_bf16": ("dk::dw_fwd_kernel", r"unsigned short"),
    # the fused pointwise backward (round 5): the streaming K = C = 64 kernel (not its lattice form,
    # a separate entry) and the fused deep kernels (32 x 32 at K = 128, 16 x 16 at K = 256)
    "dk_pwconv_bwd_bnbwd_f32": [("dk::pws::bwd_fused_kernel", r", false>$"), ("dk::pwd::bwd_kernel", ""),
                                ("dk::pwd::bwd16_kernel", "")],
    "dk_dwconv_bwd_bnbwd_f32": ("dk::dw_bwd_fused_kernel", r"^dk::dw_bwd_fused_kernel<\w+, \w+, \w+, false, float"),
    "dk_dwconv_fwd_ex_f32": ("dk::dw_fwd_kernel", r"float, false>"),
    "dk_conv2d_fwd_narrow_f32": ("dk::nar::fwd_kernel", ""),
    "dk_conv2d_wgrad_bnbwd_narrow_f32": ("dk::nar::wgrad_kernel", ""),
}


# Read / write stream counts of an entry point's dominant traffic (for the measured ceiling of
# that mix, dk_debug_stream_mix): dk_pwconv_dgrad_bnbwd_f32 reads g, the following BN's input and
# the input BN's raw input, and writes dy and dx.
ENTRY_MIX = {"dk_pwconv_dgrad_bnbwd_f32": (3, 2), "dk_pwconv_fwd_ex_f32": (1, 1), "dk_pwconv_wgrad_bnx_f32": (2, 0),
             "dk_pwconv_bwd_bnbwd_f32": (3, 1),
             "dk_dwconv_bwd_bnbwd_f32": (3, 1), "dk_dwconv_fwd_ex_f32": (1, 1), "dk_bn_add_f32": (2, 1)}


def stream_ceiling(entry):
    """The achievable HBM rate for `entry`'s read/write mix, measured now on this GPU with the
    float4 streaming probe (dk_debug_stream_mix, 205 MB per stream, 2048 x 256 threads): the
    practical peak a memory-bound kernel with that mix can reach (8 TB/s is the spec)."""
    import torch
    from dorknet_amd._hip import lib
    mix = ENTRY_MIX.get(entry)
    if mix is None:
        return None
    nin, nout = mix
    n = 256 * 56 * 56 * 64
    bufs = [torch.empty(n, device="cuda").fill_(1.0) for _ in range(nin + nout)] + [None] * 5
    p = [b.data_ptr() if b is not None else 0 for b in bufs]
    ins, outs = p[:nin] + [0] * (3 - nin), p[nin:nin + nout] + [0] * (2 - nout)
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: lib.dk_debug_stream_mix(ins[0], ins[1], ins[2], outs[0], outs[1], nin, nout, n, 2048, st)
    for _ in range(3):
        f()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in ev:
        a.record()
        f()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)[5] * 1e-3
    del bufs
    return {"value": round((nin + nout) * n * 4 / t / 1e9, 1), "unit": "GB/s", "reads": nin, "writes": nout,
            "probe": "dk_debug_stream_mix: float4 streams of 205 MB, median of 10"}


def pmc_candidates(config):
    """The committed PMC summaries of bench config `config`, newest first, in the order they were
    added to profiles/pmc_index.json (scripts/pmc_summary.py --add): commit order, not file names."""
    path = os.path.join(ROOT, "profiles", "pmc_index.json")
    if not os.path.exists(path):
        return []
    with open(path) as f:
        idx = json.load(f)
    return [os.path.join(ROOT, e["file"]) for e in reversed(idx.get("entries", [])) if e.get("config") == config]


def pmc_traffic(entry, path, config=3):
    """Average HBM bytes per dispatch of `entry`'s kernels from a committed PMC summary (`path`, or
    the newest summary of this config in profiles/pmc_index.json that has them), or (None, None)."""
    kern = ENTRY_KERNEL.get(entry)
    if not kern:
        return None, None
    cands = [path] if path else pmc_candidates(config)
    pats = kern if isinstance(kern, list) else [kern if isinstance(kern, tuple) else (kern, "")]
    for p in cands:
        if not p or not os.path.exists(p):
            continue
        with open(p) as f:
            d = json.load(f)
        n = t = 0
        for name, v in d.get("kernels", {}).items():
            if any((name.startswith(pre + "<") or name == pre) and re.search(sub, name) for pre, sub in pats):
                n += v["dispatches"]
                t += v["traffic_bytes"] * v["dispatches"]
        if n:
            return t / n, os.path.relpath(p, ROOT)
    return None, None


def attach_traffic(roof, entry, path, config):
    traffic, src = pmc_traffic(entry, path, config)
    if traffic is not None:
        roof["traffic"] = round(traffic / 1e6, 2)
        roof["traffic_unit"] = "MB per launch (HBM, rocprofv3 2*FETCH_SIZE + WRITE_SIZE)"
        roof["traffic_source"] = src


def cpu_info():
    """(model name, physical cores, logical CPUs) of this host, from lscpu."""
    import subprocess
    model, cores_per_socket, sockets, logical = None, None, None, os.cpu_count()
    try:
        out = subprocess.run(["lscpu"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                             timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "Model name":
                model = v
            elif k == "Core(s) per socket":
                cores_per_socket = int(v)
            elif k == "Socket(s)":
                sockets = int(v)
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    phys = cores_per_socket * sockets if cores_per_socket and sockets else None
    return model, phys, logical


def cpu_baseline(batch, steps=10, warmup=2):
    """Reference CPU path (restated, oracle/cpu_path.py: C/OpenMP versions of its Cython kernels
    + numpy BLAS) on `batch` images per step, timed per BASELINE.md section 3: every core this
    process may use (the GPU box gives one GPU's job a 16-CPU share: OMP_NUM_THREADS=16 and the
    affinity mask; the whole-machine physical core count is reported beside it),
    OMP_MAX_ACTIVE_LEVELS=1 (the reference's nested pranges serialised, as libgomp does by
    default), `warmup` untimed steps, then the median of `steps` timed steps."""
    import numpy as np
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cores = int(os.environ.get("OMP_NUM_THREADS", avail))
    cores = max(1, min(cores, avail))
    os.environ["OMP_NUM_THREADS"] = str(cores)
    os.environ["OMP_MAX_ACTIVE_LEVELS"] = "1"
    from threadpoolctl import threadpool_limits
    from oracle import models
    from oracle.net import OSGDMomentum
    from examples.resnet18_depsep import synthetic_batch
    from oracle._clib import lib as oracle_lib
    got = oracle_lib().oracle_set_threads(cores)
    if got != cores:
        raise RuntimeError("cpu_baseline: asked for {} OpenMP threads, got {}".format(cores, got))
    times = []
    with threadpool_limits(limits=cores):
        net = models.resnet18_depsep(backend="cy", rng=np.random.RandomState(0))
        sgd = OSGDMomentum(net, 0.05 * batch / 200.0, 0.9)
        X, _, onehot = synthetic_batch(batch, seed=0)
        for i in range(warmup + steps):
            t0 = time.perf_counter()
            net.forward(X, onehot)
            net.backward()
            sgd.update_weights()
            if i >= warmup:
                times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    model, phys, logical = cpu_info()
    return {"value": round(batch / med, 3), "unit": "images/s", "cores": cores, "kind": "port",
            "cpu_model": model, "host_physical_cores": phys, "host_logical_cpus": logical,
            "omp": {"OMP_NUM_THREADS": cores, "OMP_MAX_ACTIVE_LEVELS": 1},
            "sample": "median of {} timed training steps (fwd+bwd+SGD-momentum; after {} untimed) on a {}-image "
                      "batch of ResNet-18-depsep 225x225 fp32 -- the reference's CPU path restated (C/OpenMP "
                      "versions of its Cython kernels, -O3 -ffast-math -fopenmp, + numpy BLAS); median step "
                      "{:.3f} s, {:.1f} s in all".format(steps, warmup, batch, med, sum(times))}


def _cpu_threads():
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", avail)), avail))
    os.environ["OMP_NUM_THREADS"] = str(cores)
    os.environ["OMP_MAX_ACTIVE_LEVELS"] = "1"
    return cores


def _timed_median(fn, steps, warmup):
    import numpy as np
    times = []
    for i in range(warmup + steps):
        t0 = time.perf_counter()
        fn()
        if i >= warmup:
            times.append(time.perf_counter() - t0)
    return float(np.median(times)), sum(times)


def cpu_baseline_mnist(steps=10, warmup=2):
    """BASELINE config 1 on the reference's CPU path restated (oracle/cpu_path.py: its Cython kernels
    in C/OpenMP + numpy BLAS): MNISTNet (MNIST_basic_convnet.py:15-69), batch 64, SGD-momentum."""
    import numpy as np
    cores = _cpu_threads()
    from threadpoolctl import threadpool_limits
    from oracle import models
    from oracle.net import OSGDMomentum
    from oracle._clib import lib as oracle_lib
    oracle_lib().oracle_set_threads(cores)
    rng = np.random.default_rng(0)
    X = rng.uniform(0, 1, (64, 1, 28, 28)).astype(np.float32)
    y = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 64)]
    with threadpool_limits(limits=cores):
        net = models.mnist_net("cy", rng=np.random.RandomState(0))
        sgd = OSGDMomentum(net, 0.01, 0.9)

        def step():
            net.forward(X, y)
            net.backward()
            sgd.update_weights()
        med, tot = _timed_median(step, steps, warmup)
    model, phys, logical = cpu_info()
    return {"value": round(64 / med, 2), "unit": "images/s", "cores": cores, "kind": "port", "cpu_model": model,
            "host_physical_cores": phys, "host_logical_cpus": logical,
            "sample": "median of {} timed MNISTNet bs=64 training steps after {} untimed, reference CPU path "
                      "restated; {:.1f} s in all".format(steps, warmup, tot)}


def cpu_baseline_conv(batch=16, steps=5, warmup=1):
    """BASELINE config 2 on the reference's CPU path restated: im2col_cy + numpy SGEMM forward,
    SGEMMs + row2im_cy backward (convolution.py:58-126), on a `batch`-image slice of the
    256 x 64 x 56 x 56 input; reported as full-size passes/s (per-image time x 256)."""
    import numpy as np
    cores = _cpu_threads()
    from threadpoolctl import threadpool_limits
    from oracle import cpu_path
    from oracle._clib import lib as oracle_lib
    oracle_lib().oracle_set_threads(cores)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((batch, 64, 56, 56)).astype(np.float32)
    dY = rng.standard_normal((batch, 64, 56, 56)).astype(np.float32)
    W = (0.01 * rng.standard_normal((64, 64, 3, 3))).astype(np.float32)
    with threadpool_limits(limits=cores):
        conv = cpu_path.CyConv("c", W, None, 1, 1)

        def step():
            conv.forward(X)
            conv.backward(dY)
        med, tot = _timed_median(step, steps, warmup)
    model, phys, logical = cpu_info()
    return {"value": round(batch / 256.0 / med, 4), "unit": "passes/s", "cores": cores, "kind": "port",
            "cpu_model": model, "host_physical_cores": phys, "host_logical_cpus": logical,
            "sample": "median of {} timed fwd+dgrad+wgrad passes on a {}-image slice (after {} untimed), scaled to "
                      "256 images; reference CPU path restated (im2col_cy/row2im_cy in C/OpenMP + numpy SGEMM); "
                      "{:.1f} s in all".format(steps, batch, warmup, tot)}


def other_config(args):
    """BASELINE configs 1, 2 and 5 (one GPU): a secondary JSON line each, same timing rules
    (warm-up, then K steps between synchronizations; inputs resident in HBM)."""
    import numpy as np
    import torch
    from dorknet_amd import perfmodel
    torch.cuda.set_device(0)
    if args.config == 1:
        from examples.mnist_convnet import MNISTNet
        from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
        np.random.seed(0)
        net = MNISTNet("mnist")
        net.to_gpu()
        sgd = SGDMomentum(net, 0.01, 0.9)
        rng = np.random.default_rng(0)
        B = args.batch
        X = torch.as_tensor(rng.uniform(0, 1, (B, 1, 28, 28)).astype(np.float32), device="cuda")
        Y = torch.as_tensor(np.eye(10, dtype=np.float32)[rng.integers(0, 10, B)], device="cuda")

        def step():
            net.forward(X, Y)
            net.backward()
            sgd.update_weights()
        flops = None
        unit, metric = "images/s", "images/sec training step, MNISTNet bs=64, 1 MI355X (reference: CPU path)"
        dtype, workload = "fp32", "MNISTNet (MNIST_basic_convnet.py:15-69) fwd+loss+bwd+SGD-momentum, BASELINE config 1"
    elif args.config == 2:
        from dorknet_amd.layers.convolution import ConvLayer
        np.random.seed(0)
        conv = ConvLayer("c", filter_block_shape=(64, 64, 3, 3), stride=1, padding=1, with_bias=False)
        conv.to_gpu()
        g = torch.Generator(device="cuda").manual_seed(0)
        B = args.batch
        X = torch.randn((B, 64, 56, 56), device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
        dY = torch.randn((B, 64, 56, 56), device="cuda", generator=g).contiguous(memory_format=torch.channels_last)

        def step():
            conv.forward(X)
            conv.backward(dY)
        flops = 3 * 2 * B * 56 * 56 * 64 * 64 * 9
        unit, metric = "passes/s", "fwd+dgrad+wgrad passes/sec, ConvLayer(64,64,3,3) s1 p1 on 256x64x56x56"
        dtype, workload = "fp32", "single 3x3 ConvLayer fwd+bwd, BASELINE config 2"
    else:
        from examples.mobilenet_stack import MobileNetStack, synthetic_input
        from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
        np.random.seed(0)
        net = MobileNetStack("mobilenet_style_bf16")
        net.to_gpu()
        sgd = SGDMomentum(net, 0.05 * args.batch / 200.0, 0.9)
        X = synthetic_input(args.batch, seed=0)
        g = torch.Generator(device="cuda").manual_seed(1)
        dY = torch.randn((args.batch, 512, 7, 7), device="cuda", generator=g).to(torch.bfloat16)
        dY = dY.contiguous(memory_format=torch.channels_last)

        def step():
            net.forward(X, None)
            net.backward(dY)
            sgd.update_weights()
        flops = None
        unit, metric = "images/s", "images/sec training step, MobileNet-style dw+pw stack bs=512 bf16, 1 MI355X"
        dtype, workload = "bf16 (activations stored bf16; pointwise GEMMs on bf16 MFMA with fp32 accumulation; " \
            "depthwise, BatchNorm and weights fp32)", "16 depthwise-separable units (dw3x3-BN-pw-BN-ReLU), " \
            "ResNet-18-depsep schedule, 64x56x56 input, fwd + bwd (given output gradient) + SGD-momentum, " \
            "BASELINE config 5"
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    breakdown, dominant = None, None
    if not args.no_roofline:
        # per-entry attribution on one single-stream step, as for config 3
        with single_stream():
            with Instrument(perfmodel.MODEL.keys()) as ins:
                step()
        summ = ins.summary()
        dominant = max(summ, key=lambda n: summ[n]["ms"])
        breakdown = {n: {"ms": round(v["ms"], 3), "calls": v["calls"],
                         "frac_of_roofline": round(v["bound_ms"] / v["ms"], 3) if v["ms"] else None}
                     for n, v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])}
        torch.cuda.synchronize()
    # value: K uninstrumented steps.  The dominant entry's live duration comes from a second run of
    # K steps with its calls bracketed by events: on config 5 the event records inside the timed
    # region cost 0.8 ms of a 7.2 ms step (8.02 vs 7.22 ms, profiles/r04f_config5_bench.json against
    # r04e_ab_bench_config5.txt) -- its step is close to host-issue bound -- where config 3's is not
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    per = elapsed / args.steps
    roof = None
    if dominant:
        ins = Instrument([dominant], reserve=(breakdown[dominant]["calls"] * args.steps + 8))
        with ins:
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
        roof = roofline_entry(dominant, ins.summary()[dominant], args.steps)
        roof["timing"] = "dominant entry timed with HIP events over a second run of the same K steps"
        attach_traffic(roof, dominant, args.pmc, args.config)
    out = {"metric": metric, "value": round((1.0 if args.config == 2 else args.batch) / per, 2), "unit": unit,
           "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * per, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
           "data": "synthetic (N(0,1) inputs and output gradients, seed 0; random-init weights)",
           "config": {"workload": workload, "global_batch": args.batch, "parallelism": "dp1"}}
    if flops:
        out["achieved_tflops"] = round(flops / per / 1e12, 2)
        out["mfma_frac"] = round(flops / per / 1e12 / perfmodel.PEAK_F32_TFLOPS, 4)
    if roof:
        out["roofline"] = roof
        out["breakdown"] = breakdown
    if args.cpu_sample and args.config in (1, 2):
        out["cpu_baseline"] = cpu_baseline_mnist() if args.config == 1 else cpu_baseline_conv()
    print(json.dumps(out), flush=True)


def spawn_ranks(args):
    """`bench.py --gpus N` (N > 1) started without a torch.distributed environment: start N
    rank processes with torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) and exit
    with its status.  Runs before anything initialises the GPU, and starts the ranks as child
    processes (no exec)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def set_knobs(args):
    """--knob KIND=V (A/B runs): library knobs set before the run."""
    if not args.knob:
        return
    from dorknet_amd._hip import lib
    for kv in args.knob:
        k, v = (int(t) for t in kv.split("="))
        if lib.dk_debug_set_gemm_config(k, v) < 0:
            raise SystemExit("unknown knob {}".format(k))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    set_knobs(args)
    if args.config != 3:
        if args.gpus != 1:
            raise SystemExit("--config {} is a one-GPU configuration".format(args.config))
        if args.config == 5 and args.batch == 256:
            args.batch = 512  # the configuration's batch
        if args.config == 1 and args.batch == 256:
            args.batch = 64
        return other_config(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus {} but WORLD_SIZE={}".format(args.gpus, world))
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a HIP device")
    # one rank per GPU; a box with fewer GPUs than ranks (a launch test) shares them, and RCCL
    # cannot put two ranks on one device, so such a run uses gloo for the gradient exchange
    shared = world > ndev
    dev_index = local_rank % ndev
    torch.cuda.set_device(dev_index)
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))

    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._tensor import as_device
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    from dorknet_amd import perfmodel

    np.random.seed(0)  # identical initial weights on every rank
    net = ResNet18("DogsImageNet225ResNet18DepSep")
    net.to_gpu()
    dp = None
    if world > 1:
        from dorknet_amd.parallel import DataParallel
        dp = DataParallel(net, batch_norm=args.bn)
    sgd = SGDMomentum(net, 0.05 * args.batch / 200.0, 0.9)
    X, _, onehot = synthetic_batch(args.batch, seed=1000 + rank)
    X, onehot = as_device(X), as_device(onehot)

    def step():
        net.forward(X, onehot)
        if dp is None:
            net.backward()
        else:
            dp.backward()
        sgd.update_weights()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()

    breakdown, dominant = None, None
    if not args.no_roofline:
        # the per-entry attribution step runs single-stream, so each entry's events bracket only
        # its own kernels
        with single_stream():
            with Instrument(perfmodel.MODEL.keys()) as ins:
                step()
        summ = ins.summary()
        dominant = max(summ, key=lambda n: summ[n]["ms"])
        tot = sum(s["ms"] for s in summ.values())
        breakdown = {n: {"ms": round(s["ms"], 3), "calls": s["calls"],
                         "frac_of_roofline": round(s["bound_ms"] / s["ms"], 3) if s["ms"] else None}
                     for n, s in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])}
        step_bound = sum(s["bound_ms"] for s in summ.values())
        breakdown["_total_instrumented_ms"] = round(tot, 3)
        breakdown["_step_roofline_bound_ms"] = round(step_bound, 3)
        barrier()

    # value: K uninstrumented steps between barriers (max over ranks)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # roofline: the dominant entry's live call durations from a second run of the same K steps with
    # its calls bracketed by HIP events on the launch stream (the event records cost ~1 % of the
    # step, so they stay out of the run that gives `value`: VERDICT r4, profiles/r04g_*)
    roof = None
    if dominant:
        ins = Instrument([dominant], reserve=(breakdown[dominant]["calls"] * args.steps + 8))
        with ins:
            for _ in range(args.steps):
                step()
            barrier()
        s = ins.summary()[dominant]
        roof = roofline_entry(dominant, s, args.steps)
        roof["timing"] = "dominant entry timed with HIP events over a second run of the same K steps"
        if roof["bound"] == "hbm":
            ceil = stream_ceiling(dominant)
            if ceil is not None:
                ceil["frac"] = round(roof["achieved"] / ceil["value"], 4)
                roof["practical_peak"] = ceil
        attach_traffic(roof, dominant, args.pmc, 3)
    value = world * args.batch * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline(args.cpu_sample, args.cpu_steps, args.cpu_warmup)
    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
               "data": "synthetic (X ~ U[-128,128) 3x225x225, random one-hot labels over 120 classes; "
                       "random-init weights, seed 0)",
               "config": {"workload": "ResNet-18-depsep 225x225 training step (fwd+loss+bwd+SGD-momentum), "
                                      "BASELINE config {}".format(3 if world == 1 else 4),
                          "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                          "parallelism": "dp{}".format(world), "batch_norm": args.bn if world > 1 else "local",
                          "grad_allreduce": (None if world == 1 else
                                             "RCCL over xGMI" if not shared else
                                             "gloo: {} ranks shared {} GPU(s) (launch test, not a scaling "
                                             "point)".format(world, ndev)),
                          "input_grad": "not computed (network.backward returns nothing, as in the reference, "
                                        "which computes the image gradient and drops it)"},
               "roofline": roof, "cpu_baseline": cpu}
        if breakdown is not None:
            out["breakdown"] = breakdown
            if breakdown["_total_instrumented_ms"]:
                out["step_roofline_frac"] = round(breakdown["_step_roofline_bound_ms"] / ms_per_step, 4)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
