#!/usr/bin/env python3
"""bench.py — AudioLCM text-to-audio hot path on MI355X: generated audio-seconds per second.

One "step" = one pass of the hot path over one batch of synthetic prompts: LCM sampler
(S DiT calls + fused LCM steps) -> VAE decode_first_stage -> BigVGAN vocoder, with the
conditioning embeddings and per-prompt seeds already resident in HBM (text encoders are
out of scope); for N>1 each rank runs its own shard of 32 prompts and the
waveforms are all-gathered over RCCL (weak scaling, BASELINE config 3).

Workload at N=1: BASELINE.json configs[1] — batch 32 AudioCaps-shaped prompts, 2 LCM steps,
10 s clips (latent 20x312, mel 80x624, 159,744 samples @16 kHz).  Weights are the seeded
synthetic recipe (no checkpoints offline).

Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement for the roofline fields.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "generated audio-sec/s (real-time factor), 2-step LCM batch=32, 1/2/4/8 GPU"
SR, HOP = 16000, 256
DTYPES = {
    "mixed": "fp16 MFMA on DiT FFN / VAE k3 / BigVGAN stage 0-2 AMP convs, bf16x3-split MFMA elsewhere "
             "(fp32 accumulate, fp32 activations; waveform rel-L2 <= 1e-3 vs fp32 reference)",
    "split": "bf16x3-split MFMA (fp32 accumulate, fp32 activations)",
    "bf16": "bf16 MFMA (fp32 accumulate, fp32 activations)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="prompts per GPU")
    ap.add_argument("--lcm-steps", type=int, default=2)
    ap.add_argument("--latent-len", type=int, default=312)
    ap.add_argument("--mode", choices=["mixed", "split", "bf16"], default="mixed",
                    help="precision policy (DESIGN.md §3): mixed = fp16 MFMA on the parity-tolerant layers + "
                         "bf16x3 elsewhere (waveform parity <= 1e-3, tests/test_gpu_models.py); split = bf16x3 "
                         "everywhere (fp32 parity); bf16 = one bf16 MFMA everywhere (misses the parity bar)")
    ap.add_argument("--also-other-mode", type=int, default=1, help="N=1: also time the other precision policies")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-clips", type=int, default=4,
                    help="prompts in each batched CPU-oracle run (a bounded sample of the configs[1] batch: ~30 s per "
                         "run on 16 EPYC 9575F threads; 32 = the whole batch, ~225 s per run)")
    ap.add_argument("--cpu-budget-s", type=float, default=150.0,
                    help="time bound for the CPU-oracle runs: a further timed run starts only while its predicted time "
                         "fits (the value is the median of those that ran, up to 3)")
    ap.add_argument("--dist-backend", default=None, help="N>1: torch.distributed backend (default nccl = RCCL)")
    ap.add_argument("--force-collective", type=int, default=0,
                    help="create the process group and run the collectives even at world 1 (one-GPU rehearsal of "
                         "the N>1 path: barrier, max-over-ranks timing and the waveform all-gather over RCCL)")
    ap.add_argument("--device-map", default=None,
                    help="N>1 rehearsal: comma-separated GPU index per LOCAL_RANK (default: GPU = LOCAL_RANK)")
    ap.add_argument("--dump-wav", default=None, help="rank 0: save the gathered waveforms of the last step (.npy)")
    ap.add_argument("--extra-configs", type=int, default=1,
                    help="N=1: also time BASELINE configs[3] (C4: B=64, 4 steps + CFG) and configs[4] (C5: B=16, "
                         "30 s decode) and report them beside the headline")
    ap.add_argument("--components", type=int, default=1,
                    help="N=1: also time the SURVEY §8(f) components at the configs[1] batch (text encoders, "
                         "log-mel front-end + Encoder1D), each with its roofline")
    return ap.parse_args()


def log(msg: str) -> None:
    """Progress to stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def visible_gpus(env=None) -> int:
    """GPUs this process may use, counted WITHOUT creating a HIP context: the length of HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when one is set (the narrowest wins), else
    torch.cuda.device_count() (which on this ROCm image enumerates devices without initialising one)."""
    env = os.environ if env is None else env
    counts = [len([d for d in env[k].split(",") if d.strip() != ""])
              for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES") if k in env]
    if counts:
        return min(counts)
    return torch.cuda.device_count()


def launch_plan(gpus: int, device_map, env, n_visible: int):
    """What `bench.py --gpus N` does before anything touches a GPU.

    Returns None when this process is itself a rank (N = 1, or started by torch.distributed.run, which sets
    WORLD_SIZE), else the rank count to spawn.  Raises ValueError on a mismatch: --gpus != WORLD_SIZE under
    torchrun, --gpus < 1, a --device-map whose length is not N, or more GPUs (or a device-map index beyond those)
    than are visible."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: need at least one GPU")
    dmap = [int(x) for x in device_map.split(",")] if device_map else None
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise ValueError(f"--gpus {gpus} but torch.distributed.run started WORLD_SIZE={world} ranks")
        if dmap is not None and len(dmap) < world:
            raise ValueError(f"--device-map {device_map} names {len(dmap)} GPUs for {world} ranks")
        return None
    if dmap is not None and len(dmap) != gpus:
        raise ValueError(f"--device-map {device_map} names {len(dmap)} GPUs for --gpus {gpus}")
    need = max(dmap) + 1 if dmap else gpus
    if need > n_visible:
        raise ValueError(f"--gpus {gpus}{' --device-map ' + device_map if dmap else ''} needs {need} GPUs, "
                         f"{n_visible} visible")
    return gpus if gpus > 1 else None


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, script: str = None) -> int:
    """--gpus N > 1 without torch.distributed.run: start the N ranks (one process per GPU) as children of this
    process through torch.distributed.run on 127.0.0.1, forwarding every flag.  This process never initialises a
    GPU and never execs; it relays the children's stdout (rank 0's JSON line is the only JSON there) and returns
    torch.distributed.run's exit status (non-zero when any rank failed)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script or os.path.abspath(__file__)] + list(argv)
    log(f"starting {n} ranks: {' '.join(cmd[1:])}")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return proc.wait()


class Heartbeat:
    """Prints a progress line every `every` seconds while a long host-side phase runs."""

    def __init__(self, what: str, every: float = 20.0):
        import threading
        self.what, self.every, self.t0 = what, every, time.perf_counter()
        self.stop = threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(self.every):
            log(f"{self.what}: {time.perf_counter() - self.t0:.0f} s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(clips: int, latent_len: int, lcm_steps: int, budget_s: float, runs_wanted: int = 3):
    """The oracle (fp32 PyTorch-CPU restatement of the reference path, pinned to the reference's fixtures) on a
    BOUNDED sample of the configs[1] workload: `clips` prompts of the benchmark batch (default 4, ~30 s of CPU work
    each on the GPU box's 16-thread share) in ONE batched sampler call followed by batched VAE decode and BigVGAN
    vocode — the same region as the GPU step, from resident conditioning and per-prompt seeds to waveforms.  One
    untimed batch-1 warm-up (pages in the code and oneDNN primitives), then up to `runs_wanted` timed runs while the
    next one's predicted time fits the remaining `budget_s`; the value is their median (BASELINE.md §4's median of
    3), the count and times are reported.  Threads: the job's CPU share (OMP_NUM_THREADS, 16 on the box), not all
    affinity cores (the box asks worker pools to stay within the share); both counts are in the line.
    `--cpu-clips 32` runs the whole benchmark batch (~225 s per run) instead."""
    from audiolcm_amd import recipe
    from oracle import alcm_oracle as O
    cores = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")  # the GPU box sets the job's CPU share here (16 per GPU)
    threads = max(1, min(cores, int(share))) if share and share.isdigit() else cores
    torch.set_num_threads(threads)
    Wd, Wv, Wg = recipe.dit_state(0), recipe.vae_state(0), recipe.bigvgan_state(0)
    ids = list(range(clips))
    ctx = torch.cat([recipe.synthetic_context(1, seed0=1000 + i) for i in ids], 0)
    xT, noise = recipe.prompt_noise(ids, lcm_steps, 20, latent_len)
    runs = []
    t_start = time.perf_counter()
    with torch.no_grad(), Heartbeat(f"cpu_baseline ({clips} prompts, {threads} threads)"):
        t0 = time.perf_counter()
        O.generate(Wd, Wv, Wg, ctx[:1], xT[:1], noise[:, :1], S=lcm_steps)  # warm-up
        log(f"cpu_baseline warm-up (1 prompt): {time.perf_counter() - t0:.1f} s")
        predict = 0.0
        while len(runs) < runs_wanted:
            left = budget_s - (time.perf_counter() - t_start)
            if runs and predict > left:
                break
            t0 = time.perf_counter()
            O.generate(Wd, Wv, Wg, ctx, xT, noise, S=lcm_steps)  # one batched call: sampler, decode, vocode
            runs.append(time.perf_counter() - t0)
            predict = max(runs)
            log(f"cpu_baseline {clips}-prompt batched run {len(runs)}: {runs[-1]:.1f} s")
    clip_s = latent_len * 2 * HOP / SR
    ts = sorted(runs)[len(runs) // 2]
    audio = clips * clip_s
    return dict(value=round(audio / ts, 4), unit="audio-s/s", cores=threads, kind="port", cpu_model=cpu_model(),
                affinity_cores=cores, prompts=clips, timed_runs=len(runs), run_seconds=[round(t, 2) for t in runs],
                sample=f"{clips} of the {32} configs[1] prompts (ids 0..{clips - 1}) in one batched call ({lcm_steps} LCM "
                       f"steps, batched VAE decode + BigVGAN), {clip_s:.3f} s clips = {audio:.1f} audio-s per run; fp32 "
                       f"torch-CPU oracle on {threads} threads ({cpu_model()}); median of {len(runs)} timed run(s) "
                       f"({', '.join(f'{t:.1f}' for t in runs)} s) after a batch-1 warm-up")


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC pass (profiles/<tag>/kernels.json,
    written by scripts/prof_summary.py from separate FETCH_SIZE / WRITE_SIZE runs of this bench)."""
    import glob
    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "*", "kernels.json")), reverse=True):
        rec = json.load(open(path)).get(kernel)
        if rec and rec.get("hbm_bytes_per_launch"):
            return dict(bytes_per_launch=round(rec["hbm_bytes_per_launch"]), source=os.path.relpath(path, HERE))
    return None


def extra_configs(pipe, a):
    """BASELINE configs[3] (C4: B=64 prompts, 4 LCM steps, batch-doubled classifier-free guidance at scale 5) and
    configs[4] (C5: B=16 latents of 30 s, VAE decode + BigVGAN only: the DiT caps at T <= 845) on one GPU,
    timed like the headline (warm-up, synchronise, K steps), each with the §8(d) model roofline fraction."""
    from audiolcm_amd import recipe, roofline as RL
    out = {}
    # C4
    B, S, T = 64, 4, 312
    ids = list(range(B))
    cond = torch.cat([recipe.synthetic_context(1, seed0=1000 + i) for i in ids], 0).cuda()
    uc = torch.cat([recipe.synthetic_context(1, seed0=900 + i) for i in ids], 0).cuda()

    def c4():
        pipe.generate(cond, seeds=ids, steps=S, latent_len=T, unconditional=uc, cfg_scale=5.0)
    # C5
    B5, T5 = 16, 936
    z5 = torch.randn((B5, 20, T5), generator=torch.Generator().manual_seed(5)).cuda()

    def c5():
        pipe.decode(z5)
    for name, fn, kw, audio in (("config4", c4, RL.CONFIGS[4], B * T * 2 * HOP / SR),
                                ("config5", c5, RL.CONFIGS[5], B5 * T5 * 2 * HOP / SR)):
        for _ in range(max(1, a.warmup)):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        roof = RL.summary(RL.path_layers(**kw))
        out[name] = dict(value=round(audio / dt, 2), unit="audio-s/s", ms_per_step=round(1e3 * dt, 2),
                         path_roofline_frac_model=round(roof["t_roof_ms"] / (1e3 * dt), 4),
                         t_roof_ms=round(roof["t_roof_ms"], 2), ideal_value=round(audio / roof["t_roof_ms"] * 1e3, 1),
                         workload=("BASELINE configs[3]: 64 prompts, 4 LCM steps, batch-doubled CFG (scale 5, "
                                   "128-row DiT calls), 9.984 s clips" if name == "config4" else
                                   "BASELINE configs[4]: 16 latents of 20x936 -> mel 80x1872 -> 479,232 samples "
                                   "(29.952 s), VAE decode + BigVGAN"))
    return out


def _component_roofline(prof, wall_s: float):
    """Roofline of one component call from its per-launch HIP events: the path figure (sum over launches of
    max(F / 2.5 PF, B / 8 TB/s) / wall), the algorithmic MFMA rate over the wall, and the dominant kernel's own
    fraction of its bound."""
    from audiolcm_amd import _hip
    pf, pb = _hip.PEAK_BF16_FLOPS, _hip.PEAK_HBM_BYTES
    flops = sum(p["flops"] for p in prof)
    roof_ms = sum(p["roof_ms"] for p in prof)
    dom = max(prof, key=lambda p: p["total_ms"])
    sec = dom["total_ms"] / 1e3
    mfma = dom["flops"] / max(dom["bytes"], 1) > pf / pb
    frac = dom["flops"] / sec / pf if mfma else dom["bytes"] / sec / pb
    return dict(path_roofline_frac_build=round(roof_ms / (1e3 * wall_s), 4), t_roof_ms=round(roof_ms, 3),
                tflop=round(flops / 1e12, 4), achieved_tflops_over_wall=round(flops / wall_s / 1e12, 1),
                kernel=dom["name"], kernel_bound="mfma" if mfma else "hbm", kernel_frac=round(frac, 4),
                kernel_share=round(dom["total_ms"] / max(sum(p["total_ms"] for p in prof), 1e-9), 4),
                launches=sum(p["launches"] for p in prof))


def components(a):
    """SURVEY §8(f) components at the configs[1] batch, timed like the headline (warm-up, synchronise, K calls),
    then one instrumented call for the roofline: f1 FrozenCLAPFLANEmbedder.encode from token ids (BERT-base +
    CLAP Projection + T5-v1.1-large, 32 prompts x 77 tokens each; ldm/modules/encoders/modules.py:567-582) and
    f4 the audio -> latent direction (NAT_mel log-mel of 32 x 159,744 samples + Encoder1D + quant_conv moments;
    NAT_mel.py:66-85, ldm/models/autoencoder1d.py encode)."""
    from audiolcm_amd import _hip, recipe
    from audiolcm_amd.mel import MelNet
    from audiolcm_amd.models import AutoencoderKL
    from audiolcm_amd.text_encoder import CLAPT5TextEncoder
    B, T = a.batch, a.latent_len
    g = torch.Generator().manual_seed(7)
    enc = CLAPT5TextEncoder.from_recipe(0, split="mixed")
    cfg = enc.cfg
    ids_b = torch.randint(1, cfg.b_vocab, (B, cfg.max_len), generator=g)
    ids_t = torch.randint(1, cfg.t_vocab, (B, cfg.max_len), generator=g)
    mel = MelNet()
    st = dict(recipe.vae_state(0))
    st.update(recipe.vae_encoder_state(0))
    vae = AutoencoderKL(split="mixed").load_state_dict(st)
    wav = (0.1 * torch.randn((B, 2 * T * HOP), generator=g)).cuda()

    def text():
        enc.encode_ids(ids_b, ids_t)

    def audio_in():
        vae.encode(mel(wav))
    out = {}
    for name, fn, unit, units in (("text_encode", text, "prompts/s", B),
                                  ("mel_vae_encode", audio_in, "audio-s/s", B * 2 * T * HOP / SR)):
        for _ in range(max(1, a.warmup)):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        _hip.profile_begin()
        fn()
        torch.cuda.synchronize()
        prof = _hip.profile_end()
        out[name] = dict(value=round(units / dt, 2), unit=unit, ms_per_call=round(1e3 * dt, 3),
                         roofline=_component_roofline(prof, dt),
                         workload=(f"{B} prompts x {cfg.max_len} tokens per tower, mixed policy (fp16 MFMA on the "
                                   f"encoder linears and attention, T5 FFN-out bf16x3)" if name == "text_encode" else
                                   f"{B} clips x {2 * T * HOP} samples -> log-mel 80x{2 * T} -> Encoder1D moments "
                                   f"20x{T} (mixed policy)"))
    del enc, vae, mel
    return out


def main():
    a = parse()
    try:
        spawn = launch_plan(a.gpus, a.device_map, os.environ,
                            visible_gpus() if "WORLD_SIZE" not in os.environ else a.gpus)
    except ValueError as e:
        log(f"error: {e}")
        sys.exit(2)
    if spawn:
        sys.exit(spawn_ranks(spawn, sys.argv[1:]))
    from audiolcm_amd import _hip, recipe
    from audiolcm_amd.distributed import all_gather_rows_async, all_reduce_max, barrier, init_from_env
    from audiolcm_amd.pipeline import AudioLCMPipeline
    import torch.distributed as dist

    from audiolcm_amd import roofline as RL
    model_roof = RL.summary(RL.path_layers(B=a.batch, S=a.lcm_steps, T=a.latent_len))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = int(a.device_map.split(",")[local]) if a.device_map else local
    rank, world, local = init_from_env(a.dist_backend, device=dev, force=bool(a.force_collective))
    coll = world > 1 or bool(a.force_collective)  # the collectives run (N > 1, or the one-GPU rehearsal)
    _hip.require_device(dev)
    B, S, T = a.batch, a.lcm_steps, a.latent_len
    pipe = AudioLCMPipeline.from_recipe(0, split=a.mode)
    ids = list(range(rank * B, (rank + 1) * B))
    cond = torch.cat([recipe.synthetic_context(1, seed0=1000 + i) for i in ids], 0).cuda()
    clip_sec = T * 2 * HOP / SR

    gathered = {}
    inflight = []  # the previous step's waveform all-gather (RCCL, async): overlaps this step's kernels

    def settle():
        while inflight:
            w = inflight.pop()
            if w is not None:
                w.wait()

    def step():
        out = pipe.generate(cond, seeds=ids, steps=S, latent_len=T)
        settle()  # at most one gather in flight
        if coll:
            gathered["wav"], work = all_gather_rows_async(out["wav"], B * world)
            inflight.append(work)
        else:
            gathered["wav"] = out["wav"]
        return out

    def timed(k, profile):
        for _ in range(a.warmup):
            step()
        settle()
        torch.cuda.synchronize()
        if coll:
            barrier()
        torch.cuda.synchronize()
        if profile:
            _hip.profile_begin()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        settle()  # the last gather is inside the timed region
        torch.cuda.synchronize()
        if coll:
            barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        prof = _hip.profile_end() if profile else []
        if coll:
            dt = all_reduce_max(dt)
        return dt, prof

    # headline: the production schedule (BigVGAN resblock chains on three streams), no per-launch events
    log(f"rank {rank}/{world}: pipeline ready, headline pass ({a.warmup} warm-up + {a.steps} timed steps)")
    dt, _ = timed(a.steps, False)
    log(f"headline {1e3 * dt / a.steps:.2f} ms/step; roofline pass")
    if a.dump_wav and rank == 0:
        import numpy as np
        np.save(a.dump_wav, gathered["wav"].float().cpu().numpy())
    value = world * B * clip_sec * a.steps / dt
    # roofline pass: the same steps with live HIP-event timing of every launch and the resblock streams
    # serialised, so a kernel's measured duration is its own (concurrent kernels would share the chip)
    pipe.vocoder.set_resblock_streams(False)
    dt_prof, prof = timed(a.steps, True)
    pipe.vocoder.set_resblock_streams(True)
    gpu_ms = sum(p["total_ms"] for p in prof)
    dom = max(prof, key=lambda p: p["total_ms"]) if prof else None
    roofline = None
    if dom:
        mfma = dom["flops"] / max(dom["bytes"], 1) > _hip.PEAK_BF16_FLOPS / _hip.PEAK_HBM_BYTES
        sec = dom["total_ms"] / 1e3
        if mfma:
            ach, peak, unit = dom["flops"] / sec / 1e12, _hip.PEAK_BF16_FLOPS / 1e12, "TFLOP/s"
        else:
            ach, peak, unit = dom["bytes"] / sec / 1e9, _hip.PEAK_HBM_BYTES / 1e9, "GB/s"
        roofline = dict(bound="mfma" if mfma else "hbm", achieved=round(ach, 2), peak=peak, unit=unit,
                        frac=round(ach / peak, 4), traffic=None, kernel=dom["name"], launches=dom["launches"],
                        avg_launch_us=round(1e3 * dom["total_ms"] / dom["launches"], 2),
                        per_launch_algorithmic=round((dom["flops"] if mfma else dom["bytes"]) / dom["launches"], 1),
                        kernel_share_of_gpu_time=round(dom["total_ms"] / max(gpu_ms, 1e-9), 4),
                        path_roofline_frac_model=round(model_roof["t_roof_ms"] / (1e3 * dt / a.steps), 4),
                        path_roofline_model=dict(
                            t_roof_ms=round(model_roof["t_roof_ms"], 3), gflop=round(model_roof["gflop"], 1),
                            gbytes=round(model_roof["gbytes"], 2),
                            ideal_value=round(B * clip_sec / model_roof["t_roof_ms"] * 1e3, 1),
                            note="SURVEY.md §8(d) model (audiolcm_amd/roofline.py): bf16 layer-boundary bytes, "
                                 "sum over layers of max(F/2.5PF, B/8TB/s); frac = t_roof / ms_per_step"),
                        path_roofline_frac_build=round(sum(p["roof_ms"] for p in prof) / (1e3 * dt), 4),
                        path_roofline_note_build="sum over this build's kernel launches of max(F/2.5PF, B/8TB/s) "
                                                 "(fp32 activations, unfused byte counts) / headline wall",
                        measured_in=f"separate timed pass of the same {a.steps} steps, per-launch HIP events on the "
                                    f"launch streams, resblock streams serialised ({1e3 * dt_prof / a.steps:.2f} "
                                    f"ms/step)")
        hb = sum(p["hbm_bytes"] for p in prof)
        hms = sum(p["hbm_ms"] for p in prof)
        if hms > 0:  # the HBM fraction of the HBM-bound subset of launches
            roofline["hbm_subset"] = dict(
                achieved=round(hb / (hms / 1e3) / 1e9, 1), peak=_hip.PEAK_HBM_BYTES / 1e9, unit="GB/s",
                frac=round(hb / (hms / 1e3) / _hip.PEAK_HBM_BYTES, 4),
                launches_per_step=round(sum(p["hbm_launches"] for p in prof) / a.steps, 1),
                ms_per_step=round(hms / a.steps, 3), share_of_gpu_time=round(hms / max(gpu_ms, 1e-9), 4),
                algorithmic_gb_per_step=round(hb / a.steps / 1e9, 3),
                note="launches whose algorithmic flops/bytes < 2.5 PF / 8 TB/s: sum of this build's algorithmic bytes "
                     "/ (sum of their event time x 8 TB/s)",
                # the same time against the §8(d) model's bytes (bf16 layer boundaries, Activation1d fused), so the
                # fraction cannot rise by moving more bytes
                model_gb_per_step=round(model_roof["hbm_bound_gbytes"], 3),
                frac_model_bytes=round(model_roof["hbm_bound_gbytes"] * 1e9 / (hms / a.steps / 1e3) /
                                       _hip.PEAK_HBM_BYTES, 4),
                path_frac_model_bytes=round(model_roof["gbytes"] * 1e9 / (dt / a.steps) / _hip.PEAK_HBM_BYTES, 4),
                note_model="frac_model_bytes: the §8(d) model's bytes of its HBM-bound layers / (the same event time x "
                           "8 TB/s); path_frac_model_bytes: all of the model's bytes / (headline wall x 8 TB/s)")
        tr = pmc_traffic(dom["name"])
        if tr:  # HBM bytes per launch from the committed PMC passes of this kernel
            roofline["traffic"] = tr["bytes_per_launch"]
            roofline["traffic_source"] = tr["source"]
    line = dict(metric=METRIC, value=round(value, 2), unit="audio-s/s",
                n_gpus=dist.get_world_size() if dist.is_initialized() else world, steps=a.steps,
                warmup=a.warmup, ms_per_step=round(1e3 * dt / a.steps, 2), higher_is_better=True, scaling="weak",
                vs_baseline=None,
                dtype=DTYPES[a.mode],
                data="synthetic (seeded recipe weights, N(0,1) conditioning, per-prompt seeds)",
                config=dict(workload=f"BASELINE configs[1]: batch={B} prompts/GPU, {S} LCM steps, "
                                     f"{clip_sec:.3f} s clips (latent 20x{T}, mel 80x{2 * T}, {2 * T * HOP} samples)",
                            global_batch=B * world, per_gpu_batch=B, lcm_steps=S, latent_len=T,
                            parallelism=f"dp{world} (prompt shards, RCCL all-gather of waveforms)",
                            dist_backend=dist.get_backend() if dist.is_initialized() else None),
                roofline=roofline)
    if world == 1 and a.extra_configs:
        log("other configs (C4, C5)")
        line["other_configs"] = extra_configs(pipe, a)
    if world == 1 and a.components:
        log("SURVEY §8(f) components (text encoders, mel + Encoder1D)")
        line["components"] = components(a)
    if world == 1 and a.also_other_mode:
        log("other precision policies")
        for other in ("mixed", "split", "bf16"):
            if other == a.mode:
                continue
            pipe.set_split(other)
            dt2, _ = timed(a.steps, False)
            line[f"{other}_mode"] = dict(value=round(B * clip_sec * a.steps / dt2, 2),
                                         ms_per_step=round(1e3 * dt2 / a.steps, 2), dtype=DTYPES[other])
        pipe.set_split(a.mode)
    if rank == 0 and world == 1 and a.cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(a.cpu_clips, T, S, a.cpu_budget_s)
    if rank == 0:
        line["kernels"] = sorted(({k: (round(v, 3) if isinstance(v, float) else v) for k, v in p.items()}
                                  for p in prof), key=lambda p: -p["total_ms"])[:8]
        if os.environ.get("ALCM_BENCH_ALL_KERNELS"):
            for p in sorted(prof, key=lambda p: -p["total_ms"]):
                print(f"{p['name'][:72]:72s} n={p['launches']:5d} {p['total_ms'] / a.steps:8.3f} ms/step "
                      f"roof {p['roof_ms'] / a.steps:7.3f}", file=sys.stderr)
        print(json.dumps(line), flush=True)
    if coll:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
