"""The TfJob workload: ``python -m k8s_amd.trainer``.

What the operator launches in every replica's ``tensorflow`` container. Its
only contract with the operator is the reference's: ``TF_CONFIG`` in the
environment (`/root/reference/pkg/trainer/replicas.go:188-203`) and the
process exit code (`/root/reference/pkg/trainer/training.go:45-73`):

* role from ``TF_CONFIG.task``: MASTER/CHIEF/WORKER ranks form the RCCL group
  (master -> rank 0, rendezvous on the master's service address); a PS task
  runs the default parameter server until the master shuts it down;
* data-parallel strategies: ``allreduce`` (bucketed RCCL all-reduce
  overlapped with backward, ``parallel/ddp.py``) or ``ps`` (sharded parameter
  service: reduce-scatter push / owner update / all-gather pull,
  ``parallel/ps.py``);
* exit codes: 0 success; 1 permanent (bad config, numerics, OOM -- the
  reference treats OOMKilled as permanent); 128+ retryable (collective /
  rendezvous / connection failures, SIGTERM): the operator restarts the
  replica and it resumes from the latest checkpoint;
* outputs (chief only): ``<logdir>/events.out.tfevents.*`` (TensorBoard),
  ``<logdir>/metrics.jsonl`` (one JSON record per logged step, plus
  ``start`` / ``step0`` / ``done`` events with wall-clock times so the
  job-create -> step0 latency can be measured), and TF-style
  ``<ckpt_dir>/model.ckpt-N`` checkpoints (``utils/checkpoint.py``);
* ``--hang-timeout S``: a watchdog exits 143 (retryable) when no step completes for S seconds (a wedged
  collective); ``--trace 1|sync`` wraps the step phases in ROCTx ranges for ``rocprofv3 --marker-trace``
  (``sync`` also logs per-phase milliseconds) -- ``utils/trace.py``. ``K8S_AMD_CHECK_NUMERICS=1`` /
  ``K8S_AMD_SYNC_OPS=1`` turn on the kernel debug checks (``utils/debug.py``).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import time
import traceback
from typing import Optional

import torch

EXIT_OK = 0
EXIT_PERMANENT = 1
EXIT_RETRYABLE = 138  # 128 + 10: >= 128 is "retryable" in the operator's exit-code contract
EXIT_SIGTERM = 143


class RetryableError(RuntimeError):
    pass


def parse(argv=None):
    from k8s_amd.models.registry import MODELS

    ap = argparse.ArgumentParser(prog="python -m k8s_amd.trainer", description="k8s_amd TfJob trainer")
    ap.add_argument("--model", default="resnet50", choices=MODELS)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=None, help="per-rank batch (default: model preset)")
    ap.add_argument("--seq", type=int, default=None)
    ap.add_argument("--image", type=int, default=None)
    ap.add_argument("--optimizer", default=None, choices=["sgd", "adam"])
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--weight-decay", type=float, default=None)
    ap.add_argument("--warmup-steps", type=int, default=0, help="linear LR warmup")
    ap.add_argument("--max-grad-norm", type=float, default=None)
    ap.add_argument("--strategy", default="allreduce", choices=["allreduce", "ps"])
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    # Both multi-GPU side-stream paths below are opt-in (the examples for configs 3/4 turn them on): they have run on
    # gloo and on 2 ranks sharing one GPU, not yet on RCCL with one rank per GPU.
    ap.add_argument("--grad-comm", default="auto", choices=["auto", "fp32", "bf16"],
                    help="gradient transport: bf16 = all-to-all reduce-scatter with fp32 accumulation (16 GB instead "
                         "of 32 GB per step on Llama-3-8B); auto = fp32")
    ap.add_argument("--zero", default="auto", choices=["auto", "0", "1"],
                    help="ZeRO-1 for --strategy allreduce: reduce-scatter + owner update (fp32 master and moments "
                         "stay 1/world per rank) + bf16 all-gather of the updated weights (same xGMI bytes as an "
                         "all-reduce; optimizer state and update pass / world per rank). auto = off")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    ap.add_argument("--mlm-head", default="gathered", choices=["gathered", "every-token"],
                    help="BERT: MLM head on the masked-position slots (the original pretraining data format) or on "
                         "every token (HF BertForPreTraining's layout; same loss and gradients, more head FLOPs)")
    ap.add_argument("--logdir", default=os.environ.get("K8S_AMD_LOGDIR", ""))
    ap.add_argument("--ckpt-dir", default=os.environ.get("K8S_AMD_CKPT_DIR", ""))
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--ps-sync-every", type=int, default=-1,
                    help="push a variable snapshot to the TfJob's PS tasks every N steps (the PS tasks are the "
                         "variable store of record; a restarted job resumes from them). -1: 100 when TF_CONFIG "
                         "has PS tasks, 0: never")
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fresh-batches", action="store_true", help="draw a new synthetic batch every step")
    ap.add_argument("--graph", action="store_true", default=os.environ.get("K8S_AMD_GRAPH", "0") == "1",
                    help="capture the whole step in a hipGraph after warmup (single rank, all-reduce strategy)")
    ap.add_argument("--fail-at-step", type=int, default=-1, help="(testing) raise a retryable failure once")
    ap.add_argument("--hang-timeout", type=float, default=float(os.environ.get("K8S_AMD_HANG_TIMEOUT", "0")),
                    help="exit 143 (retryable) when no step completes for this many seconds (0: off)")
    ap.add_argument("--hang-at-step", type=int, default=-1, help="(testing) stall forever at this step")
    ap.add_argument("--trace", default=os.environ.get("K8S_AMD_TRACE", ""), choices=["", "0", "1", "sync"],
                    help="ROCTx ranges per step phase (rocprofv3 --marker-trace); 'sync' also logs phase_ms")
    return ap.parse_args(argv)


# resnet50: the headline config's per-GPU batch (bench.py --batch default), so the TfJob path and the bench run the
# same thing. Transformers sized for the 288 GB HBM (one MI355X, round 5, profiles/r05_transformer_batch.jsonl):
# BERT-base s128 676k tok/s at 64 -> 930k at 256 -> 1.03M at 512 -> 1.06M at 1024 (41 GB); Llama-3-8B s4096
# 17.9k at 1 -> 20.1-20.5k at 2 -> 21.7k at 4 (211 GB peak)
_DEFAULT_BATCH = {"resnet50": 3072, "resnet_tiny": 8, "bert_base": 1024, "bert_tiny": 4, "llama3_8b": 4,
                  "llama_1b": 4, "llama_tiny": 2}


def _process_start_time() -> Optional[float]:
    """Wall-clock start of this process (age from /proc/self/stat starttime vs /proc/uptime, 10 ms resolution): the
    interpreter and import time before train() runs is part of create -> step 0 and is reported apart from it."""
    try:
        with open("/proc/self/stat") as f:
            ticks = int(f.read().rsplit(")", 1)[1].split()[19])  # field 22 of stat(5); the split starts at field 3
        with open("/proc/uptime") as f:
            up = float(f.read().split()[0])
        return time.time() - (up - ticks / os.sysconf("SC_CLK_TCK"))
    except (OSError, ValueError, IndexError):
        return None


class _Metrics:
    def __init__(self, logdir: str, enabled: bool):
        self.enabled = enabled and bool(logdir)
        self.tb = None
        self.f = None
        if self.enabled:
            from k8s_amd.utils.tfevents import EventWriter

            os.makedirs(logdir, exist_ok=True)
            self.tb = EventWriter(logdir)
            self.f = open(os.path.join(logdir, "metrics.jsonl"), "a")

    def event(self, **rec):
        rec.setdefault("time", time.time())
        line = json.dumps(rec)
        print(line, flush=True)
        if self.f:
            self.f.write(line + "\n")
            self.f.flush()

    def scalars(self, step, values):
        if self.tb:
            self.tb.scalars(step, values)
            self.tb.flush()

    def close(self):
        if self.tb:
            self.tb.close()
        if self.f:
            self.f.close()


def _shutdown_ps(tf_config: Optional[str]):
    """The master tells the PS tasks to stop once training is done (real trainers exit 0 on all ranks)."""
    if not tf_config:
        return
    from k8s_amd.parallel.dist import resolve
    from k8s_amd.ps_server.grpc_tensorflow_server import call

    cluster = json.loads(tf_config).get("cluster", {})
    for addr in cluster.get("ps", []):
        for _ in range(20):
            try:
                call(resolve(addr), {"op": "shutdown"}, timeout=5)
                break
            except OSError:
                time.sleep(0.5)


def _wait_for_ps(tf_config: Optional[str], timeout: float = 120.0):
    """Liveness rendezvous with the PS tasks (the reference's workers block until the PS gRPC servers
    answer); raises RetryableError when they never come up."""
    if not tf_config:
        return
    from k8s_amd.parallel.dist import resolve
    from k8s_amd.ps_server.grpc_tensorflow_server import call

    end = time.time() + timeout
    for addr in json.loads(tf_config).get("cluster", {}).get("ps", []):
        while True:
            try:
                if call(resolve(addr), {"op": "ping"}, timeout=5).get("ok"):
                    break
            except OSError:
                pass
            if time.time() > end:
                raise RetryableError("PS task %s unreachable" % addr)
            time.sleep(0.2)


def _run_ps(info, tf_config: str) -> int:
    from k8s_amd.ps_server.grpc_tensorflow_server import serve

    cluster = json.loads(tf_config).get("cluster", {})
    return serve(cluster, "ps", info.role_index)


def _restore(a, w, opt, dev, chief: bool, world: int, metrics, psv=None, svc=None) -> int:
    """Resume from the newest of: the chief's latest checkpoint, the PS tasks' latest committed variable snapshot
    (``parallel/ps_vars.py``); returns the first step to run (0 without either)."""
    from k8s_amd.utils import checkpoint as ckpt

    meta_t = torch.tensor([-1, 0], dtype=torch.int64)  # [restored step or -1, optimizer step]
    tensors, flat = {}, None
    base = source = None
    if chief and a.ckpt_dir:
        base = ckpt.latest_checkpoint(a.ckpt_dir)
        if base:
            step0, tensors, meta = ckpt.load(base)
            meta_t[0], meta_t[1] = step0, int(meta.get("optim_step", step0 + 1))
            source = "checkpoint"
    if chief and psv is not None:
        try:
            v, meta = psv.latest()
            if v > int(meta_t[0]) and meta.get("total") == w.store.total:
                pulled = psv.pull(v)  # meta_t / source change only once the whole snapshot is in hand
                flat = pulled
                meta_t[0], meta_t[1] = v, int(meta.get("optim_step", v + 1))
                source = "ps"
        except (OSError, RuntimeError, ValueError, KeyError) as e:  # PS unreachable / no whole snapshot
            metrics.event(event="warning", message="PS variable snapshot unavailable, using the checkpoint (if "
                          "any): %s" % e)
    if world > 1:
        mt = meta_t.to(dev)
        torch.distributed.broadcast(mt, 0)
        meta_t = mt.cpu()
    step0 = int(meta_t[0])
    if step0 < 0:
        return 0

    def bcast(t: torch.Tensor):
        if world > 1:
            torch.distributed.broadcast(t, 0)

    if chief and flat is not None:
        w.store.master.copy_(flat["params"].to(w.store.master.device))
    elif chief:
        w.store.load_state_dict({k[len("params/"):]: v for k, v in tensors.items() if k.startswith("params/")})
    bcast(w.store.master)
    w.store.refresh_lowp()
    for name, buf in w.model.named_buffers():
        key = "buffers/" + name
        if chief and flat is not None and key in flat:
            buf.copy_(flat[key].view(buf.shape))
        elif chief and key in tensors:
            buf.copy_(tensors[key])
        bcast(buf)
    if svc is not None and svc.sharded:  # ZeRO-1: every rank receives only the slices it owns
        src = None
        if chief:
            src = {}
            for attr, key in opt.STATE.items():
                t = flat.get("optim/" + key) if flat is not None else tensors.get("optim/" + key)
                full = torch.zeros(w.store.total, dtype=torch.float32)
                if t is not None:
                    t = t.reshape(-1)
                    full[:t.numel()].copy_(t[:w.store.total])
                src[attr] = full
        svc.scatter_state(src, src=0)
        opt.step_count = int(meta_t[1])
        metrics.event(event="restored", source=source if chief else None,
                      checkpoint=os.path.basename(base) if (base and source == "checkpoint") else None, step=step0)
        return step0 + 1
    osd = {"step": int(meta_t[1])}
    for attr, key in opt.STATE.items():
        full = torch.zeros(w.store.total, dtype=torch.float32, device=dev)
        src = None
        if chief and flat is not None:
            src = flat.get("optim/" + key)
        elif chief:
            src = tensors.get("optim/" + key)
        if src is not None:
            src = src.reshape(-1)
            full[:src.numel()].copy_(src)
        bcast(full)
        osd[key] = full
    opt.load_state_dict(osd)
    metrics.event(event="restored", source=source if chief else None,
                  checkpoint=os.path.basename(base) if (base and source == "checkpoint") else None, step=step0)
    return step0 + 1


def train(a) -> int:
    from k8s_amd.models.registry import build
    from k8s_amd.ops.optim import FusedAdam, FusedSGD
    from k8s_amd.parallel import dist as kdist
    from k8s_amd.parallel.ddp import GradReducer
    from k8s_amd.parallel.ps import ShardedParameterService
    from k8s_amd.utils import checkpoint as ckpt
    from k8s_amd.utils.trace import Tracer, Watchdog

    t_start = time.time()
    t_proc = _process_start_time()
    tf_config = os.environ.get("TF_CONFIG")
    info = kdist.rank_from_env()
    if info is not None and info.role == "ps" and tf_config:
        return _run_ps(info, tf_config)
    use_cuda = a.device == "cuda" or (a.device == "auto" and torch.cuda.is_available())
    if a.device == "cuda" and not torch.cuda.is_available():
        print("error: --device cuda but no GPU is visible", file=sys.stderr)
        return EXIT_PERMANENT
    try:
        info = kdist.init_process_group(info, backend=("nccl" if use_cuda else "gloo"))
    except (RuntimeError, OSError, ValueError) as e:  # rendezvous trouble is transient
        raise RetryableError("process group init failed: %s" % e) from e
    rank, world = max(info.rank, 0), info.world_size
    chief = rank == 0
    dev = torch.device("cuda", info.device_index) if use_cuda else torch.device("cpu")
    torch.manual_seed(a.seed + rank)
    if chief:
        _wait_for_ps(tf_config)
    from k8s_amd.models.registry import MODEL_OPTIMIZER
    from k8s_amd.parallel.flat import ALIGN

    batch = a.batch or _DEFAULT_BATCH[a.model]
    opt_name = a.optimizer or MODEL_OPTIMIZER[a.model]
    zero = a.zero == "1"
    sharded = a.strategy == "ps" or (zero and world > 1)
    comm = a.grad_comm if a.grad_comm != "auto" else "fp32"
    metrics = _Metrics(a.logdir, chief)
    metrics.event(event="start", rank=rank, world=world, role=info.role, model=a.model, strategy=a.strategy,
                  device=str(dev), start_time=t_start, process_start_time=t_proc, zero1=bool(sharded and world > 1), grad_comm=comm,
                  optimizer=opt_name, batch=batch)

    # the sharded parameter service needs the flat buffers divisible into world equal 64-aligned shards
    w = build(a.model, dev, batch, seq=a.seq, image=a.image, seed=a.seed, fixed_batch=not a.fresh_batches,
              pad_to=world * ALIGN if sharded else ALIGN, data_seed=a.seed * 7919 + rank,
              mlm_every_token=a.mlm_head == "every-token")
    lr = a.lr if a.lr is not None else w.lr
    if opt_name == "sgd":
        wd = 5e-5 if a.weight_decay is None else a.weight_decay
        opt = FusedSGD(w.store, lr=lr, momentum=0.9, weight_decay=wd, max_grad_norm=a.max_grad_norm)
    else:
        wd = 0.01 if a.weight_decay is None else a.weight_decay
        opt = FusedAdam(w.store, lr=lr, weight_decay=wd, max_grad_norm=a.max_grad_norm)
    if world > 1:  # identical initial weights everywhere
        torch.distributed.broadcast(w.store.master, 0)
        w.store.refresh_lowp()
    comm_dtype = torch.bfloat16 if comm == "bf16" else torch.float32
    if sharded:
        svc = ShardedParameterService(w.store, opt, bucket_mb=a.bucket_mb, comm_dtype=comm_dtype)
        begin, finish = svc.begin_step, (lambda lr_: svc.step(lr=lr_))
    else:
        red = GradReducer(w.store, bucket_mb=a.bucket_mb, comm_dtype=comm_dtype)
        begin = red.begin_step

        def finish(lr_):
            red.finish()
            opt.step(grad_scale=red.grad_scale, lr=lr_)
        svc = None

    # ---- restore: only the chief reads the checkpoint (--ckpt-dir may be pod-local), then every tensor and the
    # start step are broadcast from it, so all ranks resume at the same step with identical weights and state
    ps_addrs = json.loads(tf_config).get("cluster", {}).get("ps", []) if tf_config else []
    sync_every = a.ps_sync_every if a.ps_sync_every >= 0 else (100 if ps_addrs else 0)
    psv = None
    if chief and ps_addrs and sync_every > 0:
        from k8s_amd.parallel.ps_vars import PsVariables

        psv = PsVariables(ps_addrs)
    start_step = _restore(a, w, opt, dev, chief, world, metrics, psv, svc)
    t_ready = time.time()  # model, optimizer and data built, checkpoint restored
    if world > 1:
        # step-0 transport self-check: one gradient bucket through the configured transport
        # (fp32 / bf16 all-reduce, ZeRO-1 push) against a plain fp32 all_reduce; the verdict is the same on every
        # rank, so all ranks exit together, with a permanent code: a wrong transport must not train
        check = (svc if svc is not None else red).self_check()
        metrics.event(event="transport_check", **check)
        if not check["ok"]:
            metrics.event(event="error", error="gradient transport self-check failed")
            return EXIT_PERMANENT

    def save(step):
        # sharded optimizer state gathered to the chief only, bucket by bucket, into host memory (collective); the
        # fp32 master made current everywhere first (the bf16 pull keeps only each rank's owned slices current)
        if svc is not None:
            svc.sync_master()
        full = svc.gather_state() if svc is not None else None
        if not chief:
            return
        tensors = {"params/" + k: v for k, v in w.store.state_dict().items()}
        tensors.update({"buffers/" + k: v for k, v in w.model.named_buffers()})
        for k, v in opt.state_dict(full).items():
            if torch.is_tensor(v):
                tensors["optim/" + k] = v
        base = ckpt.save(a.ckpt_dir, step, tensors, meta={"model": a.model, "optim_step": opt.step_count,
                                                          "world": world})
        metrics.event(event="checkpoint", step=step, path=base)

    def ps_push(step):
        """Variable snapshot to the PS tasks (collective for the sharded optimizer state, like save())."""
        if svc is not None:
            svc.sync_master()
        full = svc.gather_state() if svc is not None else None
        if psv is None:
            return
        snap = {"params": w.store.master}
        snap.update({"buffers/" + k: v for k, v in w.model.named_buffers()})
        fresh = set()
        for k, v in opt.state_dict(full).items():
            if torch.is_tensor(v):
                snap["optim/" + k] = v
                if full is not None:
                    fresh.add("optim/" + k)  # gathered host copies: pushed without another host copy
        psv.push(step, snap, meta={"optim_step": opt.step_count, "total": w.store.total, "model": a.model},
                 fresh=fresh)

    sync = torch.cuda.synchronize if use_cuda else (lambda: None)
    tracer = Tracer(enabled=a.trace not in ("", "0"), sync=(a.trace == "sync"), sync_fn=sync)
    # the first step includes kernel autotuning / vendor-library tuning: the watchdog starts after it
    watchdog = Watchdog(a.hang_timeout) if a.hang_timeout > 0 else None
    graph = None
    from k8s_amd.utils import debug as kdebug

    debug_on = any(kdebug.enabled_flags())
    if a.graph and use_cuda and world == 1 and a.strategy == "allreduce" and not tracer.enabled and not debug_on:
        from k8s_amd.utils.graph import StepGraph

        def body(inputs, lr_):
            begin()
            loss_ = w.loss(inputs)
            loss_.backward()
            finish(lr_)
            return loss_

        graph = StepGraph(body, opt, warmup=2)
    elif a.graph:
        metrics.event(event="warning", message="--graph needs one GPU rank, --strategy allreduce, no --trace "
                      "and no kernel debug mode")
    t_last, n_last = time.time(), 0
    loss_v = float("nan")
    try:
        for step in range(start_step, a.steps):
            if step == a.fail_at_step and a.ckpt_dir:
                marker = os.path.join(a.ckpt_dir, ".injected_failure.%d" % rank)
                if not os.path.exists(marker):
                    os.makedirs(a.ckpt_dir, exist_ok=True)
                    open(marker, "w").close()
                    raise RetryableError("injected failure at step %d" % step)
            if step == a.hang_at_step:
                time.sleep(1e9)  # (testing) a stalled collective
            cur_lr = lr * min(1.0, (step + 1) / a.warmup_steps) if a.warmup_steps else lr
            if graph is not None:
                loss = graph(w.batch(step), cur_lr)
            else:
                with tracer.phase("step"):
                    begin()
                    with tracer.phase("data"):
                        inputs = w.batch(step)
                    with tracer.phase("forward"):
                        loss = w.loss(inputs)
                    with tracer.phase("backward"):
                        loss.backward()
                    with tracer.phase("reduce+update"):
                        finish(cur_lr)
            n_last += 1
            if watchdog is not None:
                if step == start_step:
                    watchdog.start()
                watchdog.kick()
            if step == start_step or (step + 1) % a.log_every == 0 or step + 1 == a.steps:
                loss_v = float(loss.detach().float().item())
                bad = not (loss_v == loss_v and abs(loss_v) != float("inf"))
                if world > 1:  # decided together: a rank that exits alone would leave its peers in a collective
                    flag = torch.tensor([1.0 if bad else 0.0], device=dev)
                    torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
                    bad = bool(flag.item() > 0)
                if bad:
                    metrics.event(event="error", step=step, error="non-finite loss")
                    return EXIT_PERMANENT
                sync()
                now = time.time()
                rate = n_last * w.units_per_step * world / max(now - t_last, 1e-9)
                if step == start_step:
                    metrics.event(event="step0", step=step, loss=loss_v, since_start=now - t_start,
                                  setup_s=round(t_ready - t_start, 4), first_step_s=round(now - t_ready, 4))
                else:
                    extra = {"phase_ms": tracer.summary_ms()} if tracer.sync else {}
                    metrics.event(event="step", step=step, loss=loss_v, lr=cur_lr,
                                  **{"%s_per_sec" % w.unit: round(rate, 2)}, **extra)
                    metrics.scalars(step, {"loss": loss_v, "%s_per_sec" % w.unit: rate, "learning_rate": cur_lr})
                t_last, n_last = now, 0
            if a.ckpt_dir and a.ckpt_every and (step + 1) % a.ckpt_every == 0 and step + 1 < a.steps:
                save(step)
            if sync_every and ps_addrs and ((step + 1) % sync_every == 0 or step + 1 == a.steps):
                ps_push(step)
    except RetryableError:
        if psv is not None:  # let the last snapshot reach the PS tasks: the restarted job resumes from it
            try:
                psv.wait()
            except Exception:  # noqa: BLE001 -- the original failure is what gets reported
                pass
        raise
    if a.ckpt_dir and a.steps > start_step:
        save(a.steps - 1)
    if psv is not None:
        psv.wait()  # the last snapshot is committed before the PS tasks are told to stop
        metrics.event(event="ps_snapshot", step=psv.pushed)
    if watchdog is not None:
        watchdog.stop()
    if svc is not None:
        svc.sync_master()
    kdist.barrier()
    from k8s_amd.ops import gemm as kgemm

    metrics.event(event="done", steps=a.steps, loss=loss_v, elapsed=time.time() - t_start, rank=rank,
                  weights_sum=float(w.store.master.double().sum().item()), gemm_fallbacks=dict(kgemm.FALLBACKS),
                  peak_mem_gb=(round(torch.cuda.max_memory_allocated(w.store.master.device) / 2**30, 1)
                               if w.store.master.is_cuda else None))
    metrics.close()
    if chief:
        _shutdown_ps(tf_config)
    kdist.destroy()
    return EXIT_OK


def _replica_processes() -> int:
    """Processes this replica runs: one per GPU it was given, when TF_CONFIG makes it a compute task (the PS and
    single-GPU replicas run in this process)."""
    if os.environ.get("K8S_AMD_REPLICA_CHILD") == "1" or "RANK" in os.environ:
        return 1
    tfc = os.environ.get("TF_CONFIG")
    if not tfc:
        return 1
    try:
        ttype = json.loads(tfc).get("task", {}).get("type", "master").lower()
    except ValueError:
        return 1
    if ttype == "ps":
        return 1
    from k8s_amd.parallel.dist import own_task_processes

    return own_task_processes(ttype)


def _run_replica_children(n: int, argv) -> int:
    """One trainer process per local GPU (LOCAL_RANK i drives visible device i), started BEFORE anything touches
    the GPU; returns the replica's exit code: 0 when every child succeeded, else a failing child's code (a
    retryable one, >= 128, wins so the operator restarts the replica). When one child fails the others get a grace
    period to finish, then SIGTERM (they would otherwise wait forever in a collective)."""
    import subprocess

    argv = list(sys.argv[1:] if argv is None else argv)
    procs = []
    for i in range(n):
        env = dict(os.environ, LOCAL_RANK=str(i), LOCAL_WORLD_SIZE=str(n), K8S_AMD_REPLICA_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, "-m", "k8s_amd.trainer"] + argv, env=env))

    def forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    signal.signal(signal.SIGTERM, forward)
    codes = [None] * n
    deadline = None
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None and p.poll() is not None:
                rc = p.returncode
                codes[i] = 128 - rc if rc < 0 else rc  # killed by signal s -> 128 + s
                if codes[i] != 0 and deadline is None:
                    deadline = time.time() + 30.0
        if deadline is not None and time.time() > deadline:
            forward(signal.SIGTERM, None)
            deadline = time.time() + 1e9
        time.sleep(0.1)
    bad = [c for c in codes if c != 0]
    if not bad:
        return EXIT_OK
    retry = [c for c in bad if c >= 128]
    return retry[0] if retry else bad[0]


def main(argv=None) -> int:
    try:
        n = _replica_processes()
    except ValueError as e:  # the operator's GPU table and this container's devices disagree: not retryable
        print("error: %s" % e, file=sys.stderr, flush=True)
        return EXIT_PERMANENT
    if n > 1:
        return _run_replica_children(n, argv)
    a = parse(argv)
    signal.signal(signal.SIGTERM, lambda *_: os._exit(EXIT_SIGTERM))
    try:
        return train(a)
    except RetryableError as e:
        print("retryable failure: %s" % e, file=sys.stderr, flush=True)
        return EXIT_RETRYABLE
    except torch.cuda.OutOfMemoryError:
        traceback.print_exc()
        return EXIT_PERMANENT  # like OOMKilled: permanent
    except (ConnectionError, TimeoutError) as e:
        print("retryable failure: %r" % e, file=sys.stderr, flush=True)
        return EXIT_RETRYABLE
    except Exception as e:  # noqa: BLE001
        msg = str(e)
        traceback.print_exc()
        if any(s in msg for s in ("NCCL", "RCCL", "Connection", "timed out", "Gloo", "gloo")):
            return EXIT_RETRYABLE
        return EXIT_PERMANENT
