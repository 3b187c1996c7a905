"""Drop-in for the reference's training CLI (train.py:73-111, :399-634) for --model raa:

    python train.py --dataset sbmrgbd --model raa --gpus 0          (one MI355X)
    python train.py --dataset sbmrgbd --model raa --gpus 0,1,2,3    (data parallel)

Same flags, same config.yaml key tree, same poly learning-rate schedule with the two SGD
parameter groups (0.01x / 10x, train.py:161-174, :538-540), same loss (BCE weighted by the
global-batch positive ratio + 0.8 L1, both outputs, :595-597), same log line
"Epoch[e](i/n):     Loss: ...      lr: ..." (:607, parsed by plot_from_log.py) and the same
per-epoch snapshot {"epoch", "model"} (:624-626, "module." keys when more than one GPU).

MI355X-native differences:
* the iteration is one HIP-graph replay of hand-written kernels (cosnet_amd.train_step);
* `--gpus a,b,...` runs one process per GPU (torch.distributed over RCCL, started here as a
  child `torch.distributed.run`) instead of single-process DataParallel; the global batch
  (config batch_size) is split over the ranks like DataParallel's scatter, BN statistics
  stay per device, the BCE positive count is all-reduced (global-batch semantics) and
  gradients are averaged with one flat all-reduce;
* `--dataset sbmrgbd` reads the SBM-RGBD tree with the reference loader's rules, frame
  preparation on the GPU (cosnet_amd/sbm_rgbd.py); its batches change size every iteration,
  so those steps run eagerly.  `--dataset synthetic` feeds seeded frame pairs
  (cosnet_amd/data.py) through the recorded-graph step.
Extra flags: --config, --dtype (bf16 default; fp32 = the reference's arithmetic),
--max-epoches / --iters-per-epoch (override config), --graph 0 (eager), --duplicate-params
(the reference's repeated group-0 entries), --snapshot-root.
"""
import argparse
import datetime
import gc
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

LOG_START, LOG_END = "##==", "==##"


def get_arguments(argv=None):
    p = argparse.ArgumentParser(description="RGB-D co-attention (MI355X)")
    p.add_argument("--is-training", action="store_true")
    p.add_argument("--learning-rate", type=float, default=0.00025)
    p.add_argument("--weight-decay", type=float, default=0.0005)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--power", type=float, default=0.9)
    p.add_argument("--dataset", type=str, default="sbmrgbd")
    p.add_argument("--random-mirror", action="store_true")
    p.add_argument("--random-scale", action="store_true")
    p.add_argument("--not-restore-last", action="store_true")
    p.add_argument("--random-seed", type=int, default=1234)
    p.add_argument("--logFile", default="log.txt")
    p.add_argument("--cuda", default=True)
    p.add_argument("--gpus", type=str, default="0")
    p.add_argument("--model", default="raa")
    # this build
    p.add_argument("--config", default=os.path.join(REPO, "config.yaml"))
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--max-epoches", type=int, default=None)
    p.add_argument("--iters-per-epoch", type=int, default=None)
    p.add_argument("--graph", type=int, default=1)
    p.add_argument("--duplicate-params", action="store_true")
    p.add_argument("--snapshot-root", default=".")
    p.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                   help="data-parallel gradient reduction dtype (bucketed, overlapped)")
    p.add_argument("--log-mem", type=int, default=1,
                   help="logMem lines around each iteration like train.py:560-621 (0: off)")
    p.add_argument("--graph-cache", type=int, default=0,
                   help="sbmrgbd: recorded steps kept per frame size (0, the default: every "
                        "batch eager).  The loader's continuous scale x crop draws give ~340 "
                        "sizes at 473x473, so 24 slots hit on ~8%% of batches and record on "
                        "~80%% (tests/test_sbm.py::test_graph_cache_policy_on_loader_sizes): "
                        "worth enabling only for data whose sizes recur")
    p.add_argument("--graph-cache-min-hits", type=int, default=2,
                   help="sbmrgbd: record a frame size on its n-th occurrence")
    p.add_argument("--gc-every-iter", type=int, default=0,
                   help="1: gc.collect() + torch.cuda.empty_cache() after every iteration as the "
                        "reference does (train.py:619-620); off by default: it costs host time "
                        "and can release pool memory a recorded step graph relies on")
    return p.parse_args(argv)


def log_mem(logger, prefix):
    """logMem of train.py:51-58: allocated / reserved ("cached") device memory of this process's
    GPU, printed and appended to the train log.  torch.cuda.memory_cached is gone from current
    torch; memory_reserved is the same quantity (the caching allocator's pool)."""
    import torch
    total = torch.cuda.get_device_properties(None).total_memory
    mem_alloc = torch.cuda.memory_allocated()
    mem_cache = torch.cuda.memory_reserved()
    msg = (prefix + " GPU: " + str(torch.cuda.current_device()) + " mem_alloc: " +
           str(mem_alloc / 1048576.0) + "MB.  mem_cache: " + str(mem_cache / 1048576.0) +
           "MB.  total: " + str(total) + "\n")
    print(msg)
    if logger:
        logger.write(msg)


def get_fullname_of_model(abbr):
    """train.py:116-139; only the raa model is built here."""
    if abbr in ("raa", "resnet_aspp_add"):
        return "resnet_aspp_add"
    if abbr in ("ori", "original_coattention_rgb", "retrain", "original_coattention_rgb_retrained",
                "ref", "refactored_coattention_rgb"):
        raise Exception(abbr, "Model not provided by this build (only raa / resnet_aspp_add)")
    raise Exception(abbr, "Invalid model name!")


def load_config(path):
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def configure_dataset_init_model(args, user_config, stamp):
    """train.py:142-157."""
    ds = user_config["train"]["dataset"].get(args.dataset)
    if ds is None:
        raise SystemExit("dataset error: %r not in %s" % (args.dataset, args.config))
    args.batch_size = int(ds["batch_size"])
    args.maxEpoches = int(args.max_epoches if args.max_epoches is not None else ds["max_epoches"])
    args.data_dir = ds.get("data_path", "")
    args.num_classes = ds.get("num_classes", 2)
    args.img_mean = tuple(float(v) for v in ds["img_mean"])
    args.full_model_name = get_fullname_of_model(args.model)
    args.restore_from = user_config["train"]["model"][args.full_model_name].get("initial_params", "")
    args.resume = ds.get("checkpoint_file") or ""
    h, w = map(int, str(ds["output_HW"]).split(","))
    args.output_HW = (h, w)
    args.iters = int(args.iters_per_epoch if args.iters_per_epoch is not None
                     else ds.get("iterations_per_epoch", 0) or 0)
    args.snapshot_dir = os.path.join(args.snapshot_root, "snapshots", args.dataset,
                                     args.full_model_name, "H%dW%d" % (h, w), stamp)
    args.subset = ds.get("subset") or None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _relaunch_data_parallel(args, argv):
    """--gpus a,b,... outside torchrun: one child process per GPU (no exec from this process)."""
    n = len([g for g in args.gpus.split(",") if g.strip() != ""])
    env = dict(os.environ)
    env["CUDA_VISIBLE_DEVICES"] = args.gpus
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def make_dataset(args, per_rank_batch, rank, dev):
    from cosnet_amd.data import SyntheticRGBDPairs
    if args.dataset == "synthetic":
        return SyntheticRGBDPairs(args.iters or 4, args.output_HW, per_rank_batch,
                                  seed=args.random_seed + 7919 * rank, img_mean=args.img_mean)
    if args.dataset == "sbmrgbd":
        from cosnet_amd.sbm_rgbd import SBMRGBD
        if not args.data_dir or not os.path.isdir(args.data_dir):
            raise SystemExit("sbmrgbd: data_path %r not found (config.yaml train.dataset.sbmrgbd)" % args.data_dir)
        return SBMRGBD(args.data_dir, 1, args.output_HW, for_training=True, batch_size=args.batch_size,
                       subset=args.subset or None, meanval=args.img_mean, seed=args.random_seed,
                       device=dev)
    raise SystemExit("dataset %r: only sbmrgbd and synthetic are provided by this build" % args.dataset)


class _SbmBatches:
    """Shuffled global batches of the SBM-RGBD dataset, this rank's share of each (the
    DataLoader(shuffle=True) + DataParallel scatter of train.py:533-534, :591).  Every rank draws
    the same permutation and crop / scale ratios (same seed), so the ranks' frames have one size."""

    def __init__(self, db, global_batch, rank, world, seed):
        import random as _random
        self.db, self.B, self.rank, self.world = db, global_batch, rank, world
        self.rng = _random.Random(seed)
        self.perm = list(range(len(db)))

    def __len__(self):
        return len(self.db) // self.B

    def epoch(self, e):
        self.rng.seed(e * 1000003 + 17)
        self.rng.shuffle(self.perm)

    def __getitem__(self, i):
        self.db._scale_ratio = self.rng.uniform(0.7, 1.3)   # next_batch (:700-702)
        self.db._crop_ratio = self.rng.uniform(0.8, 1)
        idx = self.perm[i * self.B:(i + 1) * self.B][self.rank::self.world]
        return self.db.collate([self.db[j] for j in idx])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = get_arguments(argv)
    ngpu = len([g for g in args.gpus.split(",") if g.strip() != ""])
    if ngpu > 1 and "WORLD_SIZE" not in os.environ:
        return _relaunch_data_parallel(args, argv)
    if "WORLD_SIZE" not in os.environ:
        os.environ["CUDA_VISIBLE_DEVICES"] = args.gpus  # train.py:423, before HIP starts

    import torch
    import torch.distributed as dist

    import cosnet_amd as C
    from cosnet_amd.checkpoint import convert_state_dict, load_checkpoint, save_snapshot
    from cosnet_amd.optim import SGD, lr_poly, reference_param_groups
    from cosnet_amd.train_step import TrainStep

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise Exception("No GPU found or Wrong gpu id, please run without --cuda")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    stamp = datetime.datetime.now().strftime("%Y%m%d_%H%M%S")
    if world > 1:  # one snapshot directory for all ranks
        obj = [stamp]
        dist.broadcast_object_list(obj, src=0)
        stamp = obj[0]
    user_config = load_config(args.config)
    configure_dataset_init_model(args, user_config, stamp)
    if args.batch_size % world or args.batch_size // world < 2:
        raise SystemExit("batch_size %d must split into >= 2 pairs per GPU over %d GPUs (train-mode "
                         "BN of the ASPP pooling branch needs 2)" % (args.batch_size, world))
    per_rank = args.batch_size // world
    is0 = rank == 0

    def say(*a):
        if is0:
            print(*a, flush=True)

    logger = None
    if is0:
        os.makedirs(args.snapshot_dir, exist_ok=True)
        log_path = os.path.join(args.snapshot_dir, "%s__%s_%s_train_log.txt" % (
            args.dataset, args.full_model_name, stamp))
        logger = open(log_path, "a")
        logger.write(LOG_START + str(args) + LOG_END + "\n")
        logger.flush()
    say("=====> Configure dataset and pretrained model:", args)

    torch.manual_seed(args.random_seed)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    model = C.build_model(dtype)
    if args.restore_from and os.path.isfile(args.restore_from):
        say("=====> Loading init weights", args.restore_from)
        model.load_state(load_checkpoint(args.restore_from)["model"])
    else:
        say("=====> no initial params at %r: seeded initialisation" % args.restore_from)
    start_epoch = 0
    if args.resume:
        if os.path.isfile(args.resume):
            say("=> loading checkpoint '%s'" % args.resume)
            ck = load_checkpoint(args.resume)
            start_epoch = int(ck.get("epoch", 0))
            model.load_state_dict(convert_state_dict(ck["model"]))
        else:
            say("=> no checkpoint found at '%s'" % args.resume)
    # encoder.main_classifier only feeds `labels`, which never reaches the loss (no gradient
    # in the reference either)
    model.encoder.main_classifier.requires_grad_(False)
    model = model.to(dev).train()
    g0, g1 = reference_param_groups(model, duplicate_params=args.duplicate_params)
    opt = SGD([g0, g1], [args.learning_rate, 10 * args.learning_rate],
              momentum=args.momentum, weight_decay=args.weight_decay)
    nparams = sum(p.numel() for p in model.parameters())
    say("Total network parameters: %d" % nparams)
    if logger:
        logger.write("Parameters: %d" % nparams)
        logger.write("\n%s\t\t%s" % ("iter", "Loss(train)\n"))
        logger.flush()

    db = make_dataset(args, per_rank, rank, dev)
    sbm = args.dataset == "sbmrgbd"
    if sbm:  # augmented frames change size every batch: eager steps
        db = _SbmBatches(db, args.batch_size, rank, world, args.random_seed)
    train_len = len(db)
    max_iter = args.maxEpoches * train_len
    step = TrainStep(model, opt, per_rank, args.output_HW, graphed=bool(args.graph) and not sbm,
                     grad_dtype=args.grad_dtype)
    cache = None
    if sbm and args.graph and args.graph_cache > 0:
        # the augmented frames change size every batch (sbm_rgbd_loader.py:700-702): one recorded
        # step per recurring size instead of ~2000 host launches per batch
        from cosnet_amd.train_step import ShapeGraphCache
        cache = ShapeGraphCache(model, opt, per_rank, grad_dtype=args.grad_dtype,
                                capacity=args.graph_cache, min_hits=args.graph_cache_min_hits)
    mem = (lambda prefix: log_mem(logger, prefix)) if (args.log_mem and is0) else (lambda prefix: None)
    step.mem_hook = mem
    say("=====> Begin to train: %d iterations per epoch, %d epochs, %d GPU(s) x %d pairs" % (
        train_len, args.maxEpoches, world, per_rank))
    t_start = time.time()
    loss_history = []
    captured = False
    pending = None

    def report(ep, it, lt, lr):
        lv = float(lt.item()) / world
        loss_history.append(lv)
        say("===> Epoch[{}]({}/{}): Loss: {:.10f}  lr: {:.5f}".format(ep, it, train_len, lv, lr))
        if logger:
            logger.write("Epoch[{}]({}/{}):     Loss: {:.10f}      lr: {:.5f}\n".format(
                ep, it, train_len, lv, lr))
            logger.flush()

    for epoch in range(start_epoch, args.maxEpoches):
        if sbm:
            db.epoch(epoch)
        else:
            db.next_batch()
        for i_iter in range(train_len):
            mem(" Start batch")
            batch = db[i_iter]
            lr = lr_poly(args.learning_rate, i_iter + epoch * train_len, max_iter, args.power, epoch)
            lrs = [0.01 * lr, 10 * lr]  # train.py:171-172
            ins = (batch["target"].to(dev), batch["search_0"].to(dev), batch["target_depth"].to(dev),
                   batch["search_0_depth"].to(dev), batch["target_gt"].unsqueeze(1).to(dev).float(),
                   batch["search_0_gt"].unsqueeze(1).to(dev).float())
            mem(" After feeding data to GPU")
            if sbm and cache is not None:
                loss = cache(*ins, lrs)
            elif sbm:
                loss = step.run_batch(*ins, lrs)
            elif not captured:
                step.load(*ins)
                opt.set_lrs(lrs)
                step.capture(warmup=1)  # this iteration runs eagerly, then the graph is recorded
                captured = True
                loss = step.loss
            else:
                step.load(*ins)
                loss = step(lrs)
            # the loss line of this iteration is printed once the NEXT iteration is queued: a
            # .item() right after the replay would block the host until the step ends, so the
            # loader's work for the next batch could not overlap the device's step (the recorded
            # step's loss lives in a buffer the next replay overwrites: keep a device copy)
            lt = loss.detach().clone()
            if world > 1:
                # the reference's loss is computed on outputs gathered from the whole global
                # batch: with equal shards (and the global BCE weight) that is the rank mean
                dist.all_reduce(lt)
            if pending is not None:
                report(*pending)
            pending = (epoch, i_iter, lt, lr)
            del batch, ins
            if args.gc_every_iter:
                gc.collect()
                torch.cuda.empty_cache()
            mem(" After GC")
        if pending is not None:
            report(*pending)
            pending = None
        (cache if cache is not None else step).sync_buffers()  # rank 0's BN buffers (DataParallel replica 0)
        if is0:
            path = os.path.join(args.snapshot_dir, "snapshot_%s_%d.pth" % (args.dataset, epoch))
            save_snapshot(path, epoch + 1, model, dataparallel_keys=world > 1)
            say("=====> saving model", path)
    hours = (time.time() - t_start) / 3600
    say(hours, "h")
    if logger:
        logger.write("total training time: {:.2f} h\n".format(hours))
        logger.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
