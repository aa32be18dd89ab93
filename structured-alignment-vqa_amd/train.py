"""Training-loop surface of models/main_itp_ddp_tar_super_node.py on the savqa engine.

Same CLI flags (argparse main:430-500), same process model (one process per GPU:
`mp.spawn(main, nprocs=ngpus)` main:517, or torchrun env vars), same step
(forward → zero_grad → label-smoothed loss (+ -MIL-NCE) → backward → Adam, main:268-378),
same per-epoch eval of the validation AND training splits (main:42-142, :380-382: argmax
hits counted on non-zero answers, divided by every sample) and the 3-float all_gather of
both metric sets (main:383-404), same checkpoint naming with the DDP
`module.` key prefix (main:425-428).

Differences (hot path only): the model is savqa_amd.AttModel (HIP kernels), the
gradient all-reduce is savqa_amd.ddp.GradReducer (RCCL, live gradients only, streamed
out of the backward) instead of DistributedDataParallel(find_unused_parameters=True),
Adam is the fused savqa_amd.optim.Adam, and the GQA tar data (when present) is
read by savqa_amd.gqa (same dataset class and items) with the padding done on the
device (savqa_amd.collate); without the files, savqa_amd.data's synthetic batches.
"""
from __future__ import annotations

import argparse
import datetime
import logging
import os

import torch
import torch.distributed as dist

from .AttModel_x3 import AttModel
from .collate import forward_inputs, pack, to_device
from .data import model_args, model_args_rel, synthetic_batch, synthetic_relation_batch
from .ddp import GradReducer
from .loss import smoothed_loss
from .optim import Adam
from .utils import AverageMeter, add_module_prefix, init_params_


def build_parser():
    p = argparse.ArgumentParser()
    p.add_argument('--data_dir_azure', type=str, default=os.environ.get('PT_DATA_DIR', './tmp'))
    p.add_argument('--batch_size', type=int, default=256)
    p.add_argument('--lr', type=float, default=0.0001)
    p.add_argument('--output_dir', type=str, default=os.environ.get('PT_OUTPUT_DIR', './tmp'))
    p.add_argument('--maxlen', type=int, default=300)
    p.add_argument('--maxlen_q', type=int, default=50)
    p.add_argument('--maxlen_v', type=int, default=49)
    p.add_argument('--hidden_size', type=int, default=512)
    p.add_argument('--hidden_size_mil', type=int, default=64)
    p.add_argument('--num_blocks', type=int, default=6)
    p.add_argument('--num_epochs', type=int, default=40)
    p.add_argument('--num_heads', type=int, default=8)
    p.add_argument('--dropout_rate', type=float, default=0.5)
    p.add_argument('--dropout_rate_mcb', type=float, default=0.1)
    p.add_argument('--topN', type=int, default=1)
    p.add_argument('--num_classes', type=int, default=914)
    p.add_argument('--num_relations', type=int, default=311)
    for flag in ('with_smooth_labeling', 'with_MILNCE_loss', 'local_debug', 'decMask', 'mcb',
                 'only_obj', 'pred_rel', 'with_loc', 'with_dec', 'with_bbox'):
        p.add_argument(f'--{flag}', action='store_true')
    p.add_argument('--log_steps', type=int, default=100)
    p.add_argument('--model_v', type=int, default=3)
    p.add_argument('--ngpus', type=int, default=-1)
    p.add_argument('--num_nodes', type=int, default=1)
    # GQA files under data_dir_azure (main:437-465 defaults); read by savqa_amd.gqa
    p.add_argument('--fea_tar_fn_train', default='gt_bua_npz.tar')
    p.add_argument('--q_tar_fn_train', default='train.tar')
    p.add_argument('--g_tar_fn_train', default='gt_bua_npz.tar')
    p.add_argument('--fea_tar_fn_val', default='gt_bua_npz.tar')
    p.add_argument('--q_tar_fn_val', default='val.tar')
    p.add_argument('--g_tar_fn_val', default='gt_bua_npz.tar')
    p.add_argument('--gt_relation_fn', default='GT_relations_dict_compsite.json')
    p.add_argument('--obj_vocab_fn', type=str, default='objects_vocab.txt')
    p.add_argument('--attr_vocab_fn', type=str, default='attributes_vocab.txt')
    p.add_argument('--bbox_bin_num', type=int, default=64)
    p.add_argument('--enc_vocab_fn', type=str, default='preprocessed/de.vocab.composite2.tsv')
    p.add_argument('--ans_vocab_fn', type=str, default='preprocessed/en.vocab.tsv')
    p.add_argument('--min_cnt', type=int, default=10)
    p.add_argument('--num_workers', type=int, default=4)
    p.add_argument('--synthetic', action='store_true',
                   help='synthetic batches even when GQA files are present')
    # synthetic-data shape (used when the GQA files are absent)
    p.add_argument('--steps_per_epoch', type=int, default=10)
    p.add_argument('--num_regions', type=int, default=36)
    p.add_argument('--num_nodes_sg', type=int, default=59)
    p.add_argument('--q_len', type=int, default=14)
    return p


def run_model(model, batch, args):
    """main:318-329: forward + the MIL-NCE terms the loss subtracts (relation term only
    when only_obj is off)."""
    if "vis_fea_mask" in batch:  # collate_fn keys (GQA reader -> device collate)
        inputs = forward_inputs(batch)
    else:
        inputs = model_args(batch) if args.only_obj else model_args_rel(batch)
    lc, lv, ls, mil, mil_rel = model(*inputs, decMask=args.decMask, mcb=args.mcb)
    return lc, lv, ls, mil, (None if args.only_obj else mil_rel)


def evaluate(model, batches, with_mil, rank, args):
    """eval(), main:42-142: (loss_meter.avg, cnt_correct, cnt). The loss is the
    label-smoothed loss (+ the MIL-NCE loss with --with_MILNCE_loss, :129-131), averaged
    over samples; cnt_correct counts argmax hits among NON-ZERO answers (:125-126) while
    cnt counts every sample (:127 `cnt += batch_size`), as the reference does."""
    model.eval()
    meter = AverageMeter()
    correct = torch.zeros((), dtype=torch.int64, device=torch.cuda.current_device())
    cnt = 0
    with torch.no_grad():
        for batch in batches:
            lc, lv, ls, mil, mil_rel = run_model(model, batch, args)
            loss, lsm = smoothed_loss(lc, lv, ls, batch["answer"], mil, with_milnce=with_mil,
                                      mil_nce_rel=mil_rel)
            B = batch["answer"].shape[0]
            meter.update(float(loss), B)
            valid = batch["answer"] != 0
            correct += ((lsm.argmax(-1) == batch["answer"]) & valid).sum()
            cnt += B
    model.train()
    return meter.avg, float(correct), float(cnt)


def gather_metrics(vals, world_size, dev):
    """main:383-404: all_gather of every rank's (loss, cnt_correct, cnt); returns (loss
    averaged over ranks, summed correct, summed cnt, accuracy)."""
    t = torch.tensor(vals, dtype=torch.float32, device=dev)
    if world_size > 1:
        gathered = [torch.zeros(3, dtype=torch.float32, device=dev) for _ in range(world_size)]
        dist.all_gather(gathered, t)
        t = torch.stack(gathered)
    else:
        t = t.unsqueeze(0)
    loss, corr, cnt = float(t[:, 0].mean()), float(t[:, 1].sum()), float(t[:, 2].sum())
    return loss, corr, cnt, (corr / cnt if cnt else 0.0)


def gqa_loaders(args, rank):
    """main:180-249 with the savqa reader: bg_class from the object vocabulary, one
    DistributedSampler'd DataLoader per split whose collate_fn packs the ragged items
    (savqa_amd.collate.pack) for one H2D copy + the device-side padding."""
    import torch.utils.data as tud
    from .gqa import GQADataset_super_node, GQADataset_super_node_rel
    cls = GQADataset_super_node if args.only_obj else GQADataset_super_node_rel  # main:207-211
    with open(os.path.join(args.data_dir_azure, args.obj_vocab_fn)) as fid:
        args.bg_class = len(fid.readlines()) + 1
    out = {}
    # Workers forked from a process whose HIP runtime (and its threads) is live can
    # inherit a held lock and stall; once the device is up they are spawned instead.
    ctx = "spawn" if args.num_workers > 0 and torch.cuda.is_initialized() else None
    for split in ("train", "val"):
        ds = cls(split, args, getattr(args, f"fea_tar_fn_{split}"),
                                   getattr(args, f"q_tar_fn_{split}"),
                                   getattr(args, f"g_tar_fn_{split}"), args.topN, args.with_loc)
        sampler = tud.distributed.DistributedSampler(ds, num_replicas=args.world_size, rank=rank)
        out[split] = tud.DataLoader(ds, batch_size=args.batch_size, num_workers=args.num_workers,
                                    drop_last=True, collate_fn=pack, sampler=sampler,
                                    pin_memory=True, multiprocessing_context=ctx)
    return out


def main(gpu_rank, args):
    rank = int(os.environ.get("RANK", gpu_rank))
    local = int(os.environ.get("LOCAL_RANK", gpu_rank))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.world_size > 1 and not dist.is_initialized():
        dist.init_process_group("nccl", rank=rank, world_size=args.world_size, device_id=dev)
    if rank == 0:
        logging.basicConfig(level=logging.INFO, format='%(asctime)s %(levelname)-8s %(message)s')
    if args.model_v != 3:
        raise NotImplementedError("only model_v=3 is on the savqa hot path")
    gqa = (not args.synthetic) and os.path.exists(
        os.path.join(args.data_dir_azure, args.q_tar_fn_train))
    if gqa:
        loaders = gqa_loaders(args, rank)
        if not args.only_obj:  # main:194-196: the categories + 'no relation'
            args.num_relations = loaders["train"].dataset.num_relations + 1
    model = AttModel(None, args.hidden_size, args.hidden_size_mil, args.num_classes, args.maxlen_q,
                     args.maxlen, args.maxlen_v, args.num_blocks, args.num_heads, args.dropout_rate,
                     args.dropout_rate_mcb, args.num_relations, args.only_obj, device=dev,
                     init=False)
    init_params_(model, seed=0)  # same seed on every rank = DDP's initial broadcast
    model.train()
    opt = Adam(model, lr=args.lr)
    reducer = GradReducer(model._arena) if args.world_size > 1 else None
    if reducer:
        model.attach_reducer(reducer, batch_size=args.batch_size)
    result = {}

    def batches(seed0, split="train"):
        if gqa:  # main:219-249: GQA reader in DataLoader workers, padding on the device
            for pk in loaders[split]:
                yield to_device(pk, dev)
            return
        for i in range(args.steps_per_epoch):
            if args.only_obj:
                yield synthetic_batch(args.batch_size, Nv=args.num_regions, Lq=args.q_len,
                                      Ns=args.num_nodes_sg, topN=args.topN,
                                      num_classes=args.num_classes, seed=seed0 + i, device=dev)
            else:  # super-node batches with the relation tensors (relation loader)
                yield synthetic_relation_batch(args.batch_size, Nv=args.num_regions,
                                               Lq=args.q_len, topN=args.topN,
                                               num_relations=args.num_relations,
                                               num_classes=args.num_classes, seed=seed0 + i,
                                               device=dev)

    for epoch in range(args.num_epochs):
        # main:261-266: both meters restart every epoch
        loss_meter, loss_rank_meter = AverageMeter(), AverageMeter()
        for i, batch in enumerate(batches(1000 * epoch + 7919 * rank)):
            if reducer:
                reducer.begin()
            lc, lv, ls, mil, mil_rel = run_model(model, batch, args)
            opt.zero_grad()
            loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil,
                                    with_milnce=args.with_MILNCE_loss, mil_nce_rel=mil_rel)
            B = batch["answer"].shape[0]
            # main:326-329 / :358-361: the MIL-NCE loss term, metered every step whether or not
            # it enters the loss (--with_MILNCE_loss)
            mil_loss = -mil.detach() - (mil_rel.detach() if mil_rel is not None else 0.0)
            loss_rank_meter.update(mil_loss, B)
            loss.backward()
            opt.step(reducer=reducer)
            # main:368: every step. The values stay device scalars (the meters' sums are device
            # tensors), so the per-step update adds no host synchronisation; they are read on
            # the log steps only.
            loss_meter.update(loss.detach(), B)
            if rank == 0 and ((i + 1) % args.log_steps == 0 or i + 1 == args.steps_per_epoch):
                # main:370-377 (its "Epoch [e/num_epochs + 1]" counter kept as the reference prints it)
                logging.info('Time %s, Epoch [%d/%d], Step [%d/%d], Loss: %s, MIL NCE Loss: %s, '
                             'Avg Loss: %s, Avg MILNCE_loss: %s', datetime.datetime.now(), epoch + 1,
                             args.num_epochs + 1, i + 1, args.steps_per_epoch, float(loss),
                             float(mil_loss), float(loss_meter.avg), float(loss_rank_meter.avg))
        if gqa and hasattr(loaders["train"].sampler, "set_epoch"):
            loaders["train"].sampler.set_epoch(epoch + 1)
        # main:380-382: eval on the validation split, then on the training split
        val = evaluate(model, batches(10 ** 6 + rank, "val"), args.with_MILNCE_loss, rank, args)
        trn = evaluate(model, batches(1000 * epoch + 7919 * rank), args.with_MILNCE_loss, rank,
                       args)
        val_loss, corr, cnt, acc = gather_metrics(val, args.world_size, dev)
        train_loss, corr_t, cnt_t, acc_t = gather_metrics(trn, args.world_size, dev)
        if rank == 0:
            result = {"epoch": epoch + 1, "train_loss": float(loss_meter.avg),
                      "train_mil_loss": float(loss_rank_meter.avg), "val_loss": val_loss,
                      "accuracy": acc, "correct": corr, "cnt": cnt,
                      "train_eval_loss": train_loss, "train_accuracy": acc_t,
                      "train_correct": corr_t, "train_cnt": cnt_t}
            logging.info('Epoch [%d/%d], Val Loss: %.5f, accuracy: %d/%d = %.4f', epoch + 1,
                         args.num_epochs, val_loss, corr, cnt, acc)
            logging.info('Epoch [%d/%d], Train Loss: %.5f, accuracy: %d/%d = %.4f', epoch + 1,
                         args.num_epochs, train_loss, corr_t, cnt_t, acc_t)
            out = os.path.join(args.data_dir_azure, args.output_dir)
            os.makedirs(out, exist_ok=True)
            sd = model.state_dict()
            torch.save(add_module_prefix(sd) if args.world_size > 1 else sd,
                       os.path.join(out, f'model_{epoch + 1}.pth'))
    if args.world_size > 1:
        dist.destroy_process_group()
    return result


def cli(argv=None):
    args = build_parser().parse_args(argv)
    if "WORLD_SIZE" in os.environ:  # torchrun
        args.world_size = int(os.environ["WORLD_SIZE"])
        return main(int(os.environ.get("LOCAL_RANK", 0)), args)
    if args.ngpus == -1:
        args.ngpus = torch.cuda.device_count()
    args.world_size = args.ngpus * args.num_nodes
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '7787')
    if args.local_debug or args.world_size <= 1:
        args.world_size = 1
        return main(0, args)
    else:
        os.environ['WORLD_SIZE'] = str(args.world_size)
        import torch.multiprocessing as mp
        mp.spawn(_spawn_main, nprocs=args.ngpus, args=(args,))


def _spawn_main(gpu_rank, args):
    os.environ['RANK'] = str(gpu_rank)
    os.environ['LOCAL_RANK'] = str(gpu_rank)
    main(gpu_rank, args)


if __name__ == "__main__":
    cli()
