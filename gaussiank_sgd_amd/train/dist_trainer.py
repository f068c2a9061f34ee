"""Distributed training entry point (``ssgd``) with the reference's CLI.

Parity: reference dist_trainer.py:23-136 -- same flags and defaults
(``--batch-size --nsteps-update --nworkers --nwpernode --dataset --dnn
--data-dir --saved-dir --lr --max-epochs --pretrain --num-steps --compressor
--density --threshold``), same log directory naming
(``logs/allreduce-<prefix>-thres-<thr/1024>kbytes/<dnn>-n<P>-bs<B>-lr<lr>-ns<n>-ds<d>``),
per-rank log file ``<host>-<rank>.log``, the epoch/iteration loop with
gradient accumulation (``optimizer.local``), clip-after-synchronize for
LSTMs, and the throughput line ``Time per iteration including communication:
%f, Speed: %f images/s``.

Launch one process per GPU: ``torchrun --nproc-per-node N -m
gaussiank_sgd_amd.train.dist_trainer ...`` (or mpirun: OMPI_* variables are
understood).  New flags: ``--synthetic`` (always on: no datasets offline),
``--amp bf16``, ``--channels-last``, ``--density-warmup/--no-density-warmup``,
``--deterministic``, ``--max-iters``, ``--compress-single-rank``.
"""
from __future__ import annotations

import argparse
import logging
import os
import time

import numpy as np
import torch

from .. import settings, utils
from ..compression import compressors
from ..parallel import distributed_optimizer as hvd
from ..settings import formatter, logger
from .trainer import DLTrainer, _support_datasets, _support_dnns, rank_checkpoint_path


def ssgd(dnn, dataset, data_dir, nworkers, lr, batch_size, nsteps_update, max_epochs, nwpernode, pretrain,
         num_steps, compressor, density, threshold, gradient_path=None, amp=None, channels_last=False,
         density_warmup=True, deterministic=False, max_iters=None, compress_single_rank=False, saved_dir=".",
         bf16_shadow=True, momentum_correction=False, k_cap_factor=None, overlap=True, dump_grad_every=None,
         metrics_dir=None, f32_matmul=None, train_samples=None, checkpoint_every=2, save_final=False,
         hip_graph=False):
    rank = hvd.rank()
    device = "cpu"
    if torch.cuda.is_available():
        torch.cuda.set_device(hvd.local_rank() % torch.cuda.device_count())
        device = "cuda"
    if f32_matmul is not None:
        from ..ops import conv1x1
        conv1x1.set_f32_matmul(f32_matmul)
    # Resume: rank 0 loads the model, momentum and its own compressor state
    # (reference dist_trainer.py:26-27 loads on rank 0 only); every other rank
    # reads ITS OWN per-rank file for its residuals / DGC velocities -- those
    # are per-rank state nobody else holds.  Weights, momentum and the schedule
    # position are then broadcast from rank 0 (below).
    own_ck = None
    if pretrain is not None and rank != 0:
        own = rank_checkpoint_path(pretrain, rank)
        if own is not None and os.path.isfile(own):
            own_ck = own
        else:
            logger.warning("rank %d: no per-rank checkpoint for %s: its residuals / velocities start from zero",
                           rank, pretrain)
    resumed = pretrain is not None
    if rank != 0:
        pretrain = None
    trainer = DLTrainer(rank, nworkers, dist=False, batch_size=batch_size, is_weak_scaling=True, ngpus=1,
                        data_dir=data_dir, dataset=dataset, dnn=dnn, lr=lr, nworkers=nworkers, prefix="allreduce",
                        pretrain=pretrain, num_steps=num_steps, device=device, amp=amp,
                        channels_last=channels_last, seed=rank, weights_dir=os.path.join(saved_dir, "weights"),
                        train_samples=train_samples, checkpoint_every=checkpoint_every)
    init = torch.tensor([trainer.get_train_epoch(), trainer.get_train_iter()], dtype=torch.int64,
                        device=trainer.device)
    init = hvd.broadcast(init, root_rank=0)
    trainer.set_train_epoch(int(init[0]))
    trainer.set_train_iter(int(init[1]))
    trainer.seek_data()
    is_sparse = density < 1

    if settings.ADAPTIVE_MERGE or settings.ADAPTIVE_SPARSE:
        from ..utils.profiler import benchmark
        seq_layernames, layerwise_times, layerwise_sizes = benchmark(trainer)
        layerwise_times = hvd.broadcast_object(list(layerwise_times), 0)
        if rank == 0:
            logger.info("layerwise backward times: %s", list(layerwise_times))
            logger.info("layerwise backward sizes: %s", list(layerwise_sizes))
        logger.info("Bencharmked backward time: %f", float(np.sum(layerwise_times)))
        logger.info("Model size: %d", int(np.sum(layerwise_sizes)))
    else:
        seq_layernames, layerwise_times = None, None

    if k_cap_factor is not None:
        compressors[compressor].kcap_factor = float(k_cap_factor)
    if dump_grad_every is not None:
        settings.DUMP_GRAD_EVERY = int(dump_grad_every)
    norm_clip = None
    if dnn == "lstm":
        norm_clip = 0.25
    elif dnn == "lstman4":
        norm_clip = 400

    optimizer = hvd.DistributedOptimizer(trainer.optimizer, named_parameters=trainer.net.named_parameters(),
                                         compression=compressors[compressor], is_sparse=is_sparse, density=density,
                                         seq_layernames=seq_layernames, layerwise_times=layerwise_times,
                                         norm_clip=None, threshold=threshold, writer=None,
                                         gradient_path=gradient_path, density_warmup=density_warmup,
                                         deterministic=deterministic, compress_single_rank=compress_single_rank,
                                         momentum_correction=momentum_correction, overlap=overlap)
    comp_state = getattr(trainer, "_pending_compression", None)
    if own_ck is not None:
        from ..utils.checkpoint import load_checkpoint
        comp_state = load_checkpoint(own_ck, map_location="cpu").get("compression")
        logger.info("rank %d: per-rank compressor state from %s", rank, own_ck)
    if comp_state:
        optimizer.load_compression_state(comp_state)
    hvd.broadcast_parameters(trainer.net.state_dict(), root_rank=0)
    # momentum arena and train_epoch / train_iter from rank 0: replicas step
    # identically and agree on the density (record size) of every bucket
    optimizer.broadcast_state(root_rank=0)
    if bf16_shadow and trainer.is_cuda:
        # bf16: weight shadows + arena gradient sinks; fp32: the kernels' weight
        # gradients straight into the arena (parallel/shadow.py)
        from ..parallel import install_bf16_shadow, install_direct_grads
        if amp == "bf16":
            install_bf16_shadow(trainer.net, optimizer)
        else:
            install_direct_grads(trainer.net, optimizer)
    trainer.update_optimizer(optimizer)
    iters_per_epoch = max(1, trainer.get_num_of_training_samples() // (nworkers * batch_size * nsteps_update))
    from ..utils.watchdog import JsonlMetrics
    metrics = JsonlMetrics(os.path.join(metrics_dir or ".", "metrics-rank%d.jsonl" % rank))
    nparams = sum(p.numel() for p in trainer.net.parameters() if p.requires_grad)
    times = []
    logger.info("max_epochs: %d", max_epochs)
    display = 40 if iters_per_epoch > 40 else max(1, iters_per_epoch - 1)
    # --hip-graph: the whole step (forward, backward, compression, update)
    # replayed as one HIP graph, as bench.py's reference-batch phases do on one
    # GPU (train/graph.py GraphedStep: lr schedule, compressor seeds, dropout
    # and the density schedule stay live; the LSTM's hidden state is carried in
    # static buffers); one process, no gradient accumulation
    graphed = None
    if hip_graph:
        if trainer.is_cuda and nworkers == 1 and nsteps_update == 1 and dnn != "lstman4":
            from .graph import GraphedStep
            graphed = GraphedStep(trainer, optimizer, norm_clip)
        else:
            logger.warning("--hip-graph needs one GPU process, --nsteps-update 1 and a fixed-shape model "
                           "(not lstman4): running eagerly")
    done = 0
    # a resumed run continues where the checkpoint stopped (max_epochs is the
    # total); the reference re-ran max_epochs epochs from wherever it resumed
    done_iters = trainer.get_train_iter() // max(1, nsteps_update) if resumed else 0
    start_epoch, first_i = divmod(done_iters, iters_per_epoch)
    for epoch in range(start_epoch, max_epochs):
        hidden = None
        if dnn == "lstm":
            hidden = trainer.net.init_hidden()
            if graphed is not None:
                graphed.reset_hidden()     # the reference re-initialises the state every epoch
        for i in range(first_i if epoch == start_epoch else 0, iters_per_epoch):
            s = time.time()
            if graphed is not None:
                graphed()
            else:
                optimizer.zero_grad()
                for j in range(nsteps_update):
                    optimizer.local = j < nsteps_update - 1 and nsteps_update > 1
                    if dnn == "lstm":
                        _, hidden = trainer.train(1, hidden=hidden)
                    else:
                        trainer.train(1)
                if norm_clip is not None:
                    optimizer.synchronize()
                    optimizer.clip_grad_norm_(norm_clip)
                trainer.update_model()
            times.append(time.time() - s)
            if i % display == 0 and i > 0:
                if trainer.is_cuda:
                    torch.cuda.synchronize()
                time_per_iter = float(np.mean(times))
                speed = batch_size * nsteps_update / time_per_iter
                logger.warning("Time per iteration including communication: %f, Speed: %f images/s", time_per_iter,
                               speed)
                # this window's counts (the optimizer keeps every window for the epoch summary)
                sel = optimizer._collect_selected() if hasattr(optimizer, "_collect_selected") else []
                per_iter_sel = float(np.mean(sel)) * len(optimizer.arena.buckets) if sel else 0.0
                ratio = optimizer.wire_compression_ratio() if hasattr(optimizer, "wire_compression_ratio") else 1.0
                metrics.write(iter=int(trainer.get_train_iter()), epoch=epoch, rank=rank, time_per_iter=time_per_iter,
                              samples_per_s=speed, samples_per_s_node=speed * nworkers,
                              density=optimizer.get_current_density(),
                              selected_per_iter=per_iter_sel,
                              compression_ratio=ratio,
                              loss=float(trainer.current_loss()),
                              hbm_gb=(torch.cuda.max_memory_allocated() / 2 ** 30) if trainer.is_cuda else 0.0)
                times = []
            done += 1
            if max_iters is not None and done >= max_iters:
                if i == iters_per_epoch - 1:
                    optimizer.increase_one_epoch()
                elif hasattr(optimizer, "log_selection_summary"):
                    optimizer.log_selection_summary()
                return _finish(trainer, optimizer, save_final)
        optimizer.increase_one_epoch()
    return _finish(trainer, optimizer, save_final)


def _finish(trainer, optimizer, save_final):
    """End of the run: with ``save_final`` every rank writes its checkpoint
    (weights, momentum, its residuals / velocities, schedule position) so the
    run can be resumed with ``--pretrain <...-rank0-epoch<e>.pth>``."""
    if save_final:
        if trainer.is_cuda:
            torch.cuda.synchronize()
        fn = trainer.save_epoch_checkpoint()
        if fn:
            logger.info("final checkpoint: %s", fn)
    return trainer, optimizer


def build_parser():
    p = argparse.ArgumentParser(description="AllReduce trainer")
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--nsteps-update", type=int, default=1)
    p.add_argument("--nworkers", type=int, default=None, help="defaults to the launched world size")
    p.add_argument("--nwpernode", type=int, default=1, help="Number of workers per node")
    p.add_argument("--dataset", type=str, default="imagenet", choices=_support_datasets)
    p.add_argument("--dnn", type=str, default="resnet50", choices=_support_dnns)
    p.add_argument("--data-dir", type=str, default="./data")
    p.add_argument("--saved-dir", type=str, default=".")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--max-epochs", type=int, default=settings.MAX_EPOCHS)
    p.add_argument("--pretrain", type=str, default=None)
    p.add_argument("--num-steps", type=int, default=35)
    p.add_argument("--compressor", type=str, default="gaussian", choices=[k for k in compressors if k])
    p.add_argument("--density", type=float, default=1)
    p.add_argument("--threshold", type=int, default=524288000)
    # MI355X build additions
    p.add_argument("--amp", type=str, default=None, choices=[None, "bf16", "fp16"])
    p.add_argument("--channels-last", action="store_true")
    p.add_argument("--no-density-warmup", action="store_true")
    p.add_argument("--deterministic", action="store_true")
    p.add_argument("--compress-single-rank", action="store_true")
    p.add_argument("--max-iters", type=int, default=None)
    p.add_argument("--momentum-correction", action="store_true",
                   help="DGC momentum correction + momentum factor masking (local momentum before sparsification)")
    p.add_argument("--k-cap-factor", type=float, default=None,
                   help="record capacity k_cap = factor * k (Gaussian-k may select more than k)")
    p.add_argument("--bucket-mb", type=float, default=None,
                   help="bucket size in MB of fp32 gradients (overrides --threshold)")
    p.add_argument("--no-overlap", action="store_true", help="exchange buckets at synchronize(), not in backward")
    p.add_argument("--dump-grad-every", type=int, default=None,
                   help="with settings.LOGGING_GRADIENTS: dump every N iterations (async D2H)")
    p.add_argument("--synthetic", action="store_true", default=True,
                   help="synthetic on-device data (always on: no datasets offline)")
    p.add_argument("--no-bf16-shadow", action="store_true",
                   help="with --amp bf16: keep plain autocast casts instead of the bf16 shadow weight arena")
    p.add_argument("--logdir-root", type=str, default="./logs")
    p.add_argument("--f32-matmul", type=str, default=os.environ.get("GKSGD_F32_MATMUL", "bf16x6"),
                   choices=["native", "bf16x6"],
                   help="fp32 convolution / linear GEMM algorithm (default: %(default)s, the same as bench.py and "
                        "the library): native = fp32 MFMA only; bf16x6 = the tuner may also pick the "
                        "fp32-accurate bf16x6 product kernels (ops/conv1x1.py set_f32_matmul)")
    p.add_argument("--train-samples", type=int, default=None,
                   help="synthetic epoch length in samples (default: the dataset's real size)")
    p.add_argument("--checkpoint-every", type=int, default=2,
                   help="save a checkpoint every N trainer epochs (reference: 2)")
    p.add_argument("--hip-graph", action="store_true",
                   help="replay the whole training step as one HIP graph (one GPU process, non-recurrent models; "
                        "what bench.py does for its reference-batch phases)")
    p.add_argument("--save-final", action="store_true",
                   help="every rank saves its checkpoint at the end of the run (resume with --pretrain)")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    hvd.init()
    nworkers = args.nworkers or hvd.size()
    batch_size = args.batch_size * args.nsteps_update
    prefix = settings.PREFIX
    if args.density < 1:
        prefix = "comp-" + args.compressor + "-" + prefix
    logdir = "allreduce-%s-thres-%dkbytes/%s-n%d-bs%d-lr%.4f-ns%d-ds%s" % (
        prefix, args.threshold / 1024, args.dnn, nworkers, batch_size, args.lr, args.nsteps_update, str(args.density))
    relative_path = os.path.join(args.logdir_root, logdir)
    utils.create_path(relative_path)
    gradient_path = None
    if settings.LOGGING_GRADIENTS:
        gradient_path = "%s/gradients/%s" % (args.saved_dir, logdir)
        utils.create_path(gradient_path)
    threshold = args.threshold
    if args.bucket_mb is not None:
        threshold = int(args.bucket_mb * 1024 * 1024 / 4)
    rank = hvd.rank()
    logfile = os.path.join(relative_path, settings.hostname + "-" + str(rank) + ".log")
    hdlr = logging.FileHandler(logfile)
    hdlr.setFormatter(formatter)
    logger.addHandler(hdlr)
    logger.info("Configurations: %s", args)
    return ssgd(args.dnn, args.dataset, args.data_dir, nworkers, args.lr, args.batch_size, args.nsteps_update,
                args.max_epochs, args.nwpernode, args.pretrain, args.num_steps, args.compressor, args.density,
                threshold, gradient_path, amp=args.amp, channels_last=args.channels_last,
                density_warmup=not args.no_density_warmup, deterministic=args.deterministic,
                max_iters=args.max_iters, compress_single_rank=args.compress_single_rank, saved_dir=args.saved_dir,
                bf16_shadow=not args.no_bf16_shadow, momentum_correction=args.momentum_correction,
                k_cap_factor=args.k_cap_factor, overlap=not args.no_overlap, dump_grad_every=args.dump_grad_every,
                metrics_dir=relative_path, f32_matmul=args.f32_matmul, train_samples=args.train_samples,
                checkpoint_every=args.checkpoint_every, save_final=args.save_final, hip_graph=args.hip_graph)


if __name__ == "__main__":
    main()
