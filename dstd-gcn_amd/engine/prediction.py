"""PredictionEngine / ModelWrapper (reference engine/prediction.py).

Same constructor, method names, arguments, return values and checkpoint
format as the reference, driving the MI355X model:

* ``train`` (:198-317): train-mode forward (native, batch-statistics BN),
  mpjpe loss, the inverse-time augmentation pass, ``all_loss / 2``, native
  backward, Adam step, StepLR at epoch end.  Losses accumulate on the GPU; the
  epoch synchronises once when it reports its average.  Under
  ``torch.distributed`` (one process per GPU) gradients are averaged with one
  flat all-reduce per step (dstd_dist.allreduce_grads) and the reported
  epoch losses are the global averages (one all-reduce of the loss sums and
  sample counts).  The engine opts the model into the in-place gradient arena
  (dstd_native.grad_sink); other callers get plain autograd gradients.
* ``test`` (:319-430): eval forward, then the per-frame MPJPE of every batch
  in one kernel (dstd_frame_mpjpe) accumulating on the device; one
  synchronisation per call instead of one ``.item()`` per frame and batch.
  Under ``torch.distributed`` with more than one rank the batches are sharded
  round-robin over the ranks (unless the loader already shards through a
  DistributedSampler) and the per-frame sums and sample counts are
  all-reduced (dstd_dist.reduce_partials), so every rank returns the metric of
  the whole loader.
* ``save`` / ``recover`` (:159-182): the same ``{"lr", "err", "model",
  "optimizer", "scheduler", "epoch"}`` dict with ``model.``-prefixed keys;
  recover loads with ``weights_only=True``.
"""
import warnings

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

import dstd_native as native

from .loss import LOSSES, AccumLoss, DeviceAccum
from .transform import TRANSFORMS


class ModelWrapper(nn.Module):
    """Model + weighted losses (prediction.py:21-104); single output."""

    def __init__(self, model, loss, n_out=1):
        super(ModelWrapper, self).__init__()
        self.model = model
        self.n_out = n_out
        if n_out != 1:
            raise NotImplementedError("ModelWrapper: multi-output models (n_out > 1) are not built")
        self.all_loss = set()
        self.loss_funcs = {}
        for ls in loss.keys():
            name = loss[ls][0]
            if name not in LOSSES:
                raise NotImplementedError(f"loss '{name}' is not built (shipped configs use jl2 only)")
            self.loss_funcs[ls] = (LOSSES[name], loss[ls][1])
            if ls in self.all_loss:
                raise ValueError("Redundant Error", ls)
            self.all_loss.add(ls)

    def forward(self, inputs, training=True):
        outputs = self.model(inputs)
        if training:
            return outputs
        return outputs[-1] if isinstance(outputs, list) else outputs

    def calc_loss(self, pred, gt, loss_type="all", wgts=None):
        if loss_type != "all" and loss_type != "sum" and loss_type not in self.all_loss:
            raise ValueError(f"Invalid loss type {loss_type}")
        if loss_type == "all":
            return {ls: w * fn(pred, gt, wgts) for ls, (fn, w) in self.loss_funcs.items()}
        if loss_type == "sum":
            loss = 0
            for fn, w in self.loss_funcs.values():
                loss = loss + w * fn(pred, gt, wgts)
            return loss
        return self.loss_funcs[loss_type]


def _world():
    """(rank, world size) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _to_dev(x, dev):
    if isinstance(x, list):
        return [t.float().to(dev, non_blocking=True) for t in x]
    return x.float().to(dev, non_blocking=True)


class PredictionEngine:

    def __init__(self, config, model, logger, device=None):
        self.model = ModelWrapper(model, config["loss"], config["n_out"])
        self.config = config
        self.logger = logger
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        self.reset()
        if config["transform"] not in TRANSFORMS:
            raise NotImplementedError(f"transform '{config['transform']}' is not built (shipped configs use tsc)")
        self.transform_func, self.inverse_func = TRANSFORMS[config["transform"]]
        logger.info("Trainable number of parameters of the network is: " +
                    str(sum(p.numel() for p in model.parameters() if p.requires_grad)))
        logger.info("Total number of parameters of the network is: " + str(sum(p.numel() for p in model.parameters())))

    def transform(self, x):
        if self.transform_func is None:
            return x
        return [self.transform_func(s) for s in x] if isinstance(x, list) else self.transform_func(x)

    def inverse(self, x):
        if self.inverse_func is None:
            return x
        return [self.inverse_func(s) for s in x] if isinstance(x, list) else self.inverse_func(x)

    def _graphed(self):
        """learn.graph: capture the training step as a HIP graph (engine/graphed.py)
        -- one process per GPU without a process group (a gloo all-reduce
        cannot be captured)."""
        return bool(self.config["learn"].get("graph", False)) and self.device.type == "cuda" and _world()[1] == 1

    def reset(self):
        self.lr = self.config["learn"]["lr"]
        self.best_err = float("inf")
        self.optimizer, self.scheduler = self._setup_learn(self.model.parameters(), self.config["learn"]["opt"])

    def recover(self, checkpoint_path, model_only=False):
        state = torch.load(checkpoint_path, map_location=self.device, weights_only=True)
        err = state["err"]
        epoch = state["epoch"]
        if not model_only:
            self.model.load_state_dict(state["model"])
            self.optimizer.load_state_dict(state["optimizer"])
            self.lr = state["lr"]
        self.logger.info("load from lr {}, curr_avg {} from {}.".format(state["lr"], err, checkpoint_path))
        return epoch, err

    def save(self, checkpoint_path, err, epoch, is_best=False):
        state = {
            "lr": self.lr,
            "err": err,
            "model": self.model.state_dict(),
            "optimizer": self.optimizer.state_dict(),
            "scheduler": self.scheduler.state_dict(),
            "epoch": epoch,
        }
        torch.save(state, checkpoint_path + "/last.pth")
        if is_best:
            torch.save(state, checkpoint_path + "/best.pth")

    def _setup_learn(self, params, opt_type="adam"):
        if opt_type != "adam":
            raise NotImplementedError(f"optimizer '{opt_type}' (shipped configs use adam)")
        if self._graphed():
            # replayable step (engine/graphed.py): device-side step count and a
            # tensor learning rate that StepLR updates in place
            optimizer = optim.Adam(params, lr=torch.tensor(float(self.config["learn"]["lr"]), device=self.device),
                                   weight_decay=self.config["learn"]["weight_decay"], capturable=True)
        else:
            # the reference's Adam (:188-192) as torch's single-kernel
            # implementation on the GPU: same update, ~30 foreach launches and
            # ~0.8 ms of host time per step fewer (scripts/train_host_probe.py)
            params = list(params)
            fused = all(p.is_cuda for p in params)
            optimizer = optim.Adam(params, lr=self.config["learn"]["lr"],
                                   weight_decay=self.config["learn"]["weight_decay"], fused=fused or None)
        self._graph_step = None
        scheduler = optim.lr_scheduler.StepLR(optimizer, step_size=self.config["learn"]["step_size"],
                                              gamma=self.config["learn"]["gamma"])
        return optimizer, scheduler

    # ------------------------------------------------------------------
    def train(self, train_loader, epoch, time_tsfm=None, scale_tsfm=None, weights=None, max_iter=-1):
        dev = self.device
        t_l = {key_loss: DeviceAccum(dev) for key_loss in self.config["loss"]}
        self.model.train()
        # backward accumulates straight into .grad (dstd_native.grad_sink) for
        # this epoch's steps only: the flag is restored on the way out, so a
        # caller that later wraps the model (DDP reducer hooks, user hooks)
        # gets ordinary autograd gradients
        net = self.model.model
        prev_inplace = getattr(net, "_dstd_inplace_grads", False)
        net._dstd_inplace_grads = True
        try:
            return self._train_epoch(train_loader, epoch, time_tsfm, scale_tsfm, weights, max_iter, t_l)
        finally:
            net._dstd_inplace_grads = prev_inplace

    def _train_epoch(self, train_loader, epoch, time_tsfm, scale_tsfm, weights, max_iter, t_l):
        dev = self.device
        distributed = _world()[1] > 1
        num_iter = len(train_loader) if max_iter == -1 else min(len(train_loader), max_iter)
        for i, (inputs, inputs_inv, targets, all_seqs) in enumerate(train_loader):
            inputs, inputs_inv, targets = _to_dev(inputs, dev), _to_dev(inputs_inv, dev), _to_dev(targets, dev)
            N = inputs[0].shape[0] if isinstance(inputs, list) else inputs.shape[0]

            def step(inp, inp_inv, targ):
                return self._step(inp, inp_inv, targ, time_tsfm, scale_tsfm, weights, distributed)

            tensors = not isinstance(inputs, list) and torch.is_tensor(inputs_inv)
            if self._graphed() and tensors:
                g = self._graph_step
                if g is None:
                    from .graphed import GraphedStep
                    g = self._graph_step = GraphedStep(step, (inputs, inputs_inv, targets), self.model.model,
                                                       self.optimizer)
                losses = g(inputs, inputs_inv, targets) if g.matches(inputs, inputs_inv, targets) else \
                    step(inputs, inputs_inv, targets)  # (a ragged last batch runs eagerly)
            else:
                losses = step(inputs, inputs_inv, targets)
            for ls, v in zip(t_l, losses):
                t_l[ls].update(v * N, N)
            if i >= num_iter - 1:
                break
        if distributed:  # global averages: one all-reduce of (loss sums, sample counts)
            from dstd_dist import reduce_partials
            sums = torch.stack([t_l[ls].sum for ls in t_l])
            counts = torch.tensor([float(t_l[ls].count) for ls in t_l], dtype=torch.float64, device=sums.device)
            sums, counts = reduce_partials(sums, counts)
            avg = {ls: float(s) / float(c) if c else 0.0 for ls, s, c in zip(t_l, sums.tolist(), counts.tolist())}
        else:
            avg = {ls: t_l[ls].avg for ls in t_l}
        desc = f"epoch: {epoch + 1}|train|" + "".join("{}:{:.2f}|".format(ls, avg[ls]) for ls in t_l)
        self.logger.info(desc)
        self.scheduler.step()
        # the reference reads get_lr() here (:311): on a StepLR boundary that is
        # the decayed rate decayed once more -- the value its checkpoints store
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            self.lr = float(self.scheduler.get_lr()[0])
        return sum(avg.values())

    def _step(self, inputs, inputs_inv, targets, time_tsfm, scale_tsfm, weights, distributed):
        """One training step (:231-294): forward (pair), losses, backward,
        gradient all-reduce / clip, Adam.  Returns the forward pass's losses
        (one per loss type, in config order) for the epoch averages."""
        if time_tsfm is not None:
            inputs = time_tsfm.transform(inputs)
        inputs = self.transform(inputs)
        # the batch and its time reversal as one native forward pair
        # (DSTDGCN.forward_pair: per-half BatchNorm statistics, so the same
        # step as the two calls of the reference, with half the launches)
        pair = self.config["inverse"] and hasattr(self.model.model, "forward_pair")
        if pair:
            if time_tsfm is not None:
                inputs_inv = time_tsfm.transform(inputs_inv)
            inputs_inv = self.transform(inputs_inv)
            out_pair = self.model.model.forward_pair(inputs, inputs_inv)
            outputs = self.inverse(out_pair[0])
        else:
            outputs = self.inverse(self.model(inputs, False))
        if scale_tsfm is not None:
            outputs = scale_tsfm.inverse(outputs)
        if time_tsfm is not None:
            outputs = time_tsfm.inverse(outputs)
        t = outputs.shape[1]
        targets_l = targets[:, -t:] if t != targets.shape[1] else targets
        loss = self.model.calc_loss(outputs, targets_l, "all", weights)
        all_loss = 0
        for ls in loss:
            all_loss = all_loss + loss[ls]
        if self.config["inverse"]:  # time-reversed augmentation pass (:267-287)
            if pair:
                outputs_inv = self.inverse(out_pair[1])
            else:
                if time_tsfm is not None:
                    inputs_inv = time_tsfm.transform(inputs_inv)
                inputs_inv = self.transform(inputs_inv)
                outputs_inv = self.inverse(self.model(inputs_inv, True))
            targets_inv = targets.flip(1)
            t = outputs_inv.shape[1]
            targets_il = targets_inv[:, -t:] if t != targets_inv.shape[1] else targets_inv
            if time_tsfm is not None:
                outputs_inv = time_tsfm.inverse(outputs_inv)
            if scale_tsfm is not None:
                outputs_inv = scale_tsfm.inverse(outputs_inv)
            loss_inv = self.model.calc_loss(outputs_inv, targets_il, "all", weights)
            for ls in loss_inv:
                all_loss = all_loss + loss_inv[ls]
            all_loss = all_loss / 2
        self.optimizer.zero_grad()
        all_loss.backward()
        if distributed:
            from dstd_dist import allreduce_grads
            allreduce_grads(self.model.parameters())
        if self.config.get("clip", -1) > 0:
            nn.utils.clip_grad_norm_(self.model.model.parameters(), max_norm=self.config["clip"])
        self.optimizer.step()
        return tuple(loss[ls].detach() for ls in self.config["loss"])

    # ------------------------------------------------------------------
    def test(self, test_loader, input_n=10, eval_frame=None, dim_used=None, joint_to_ignore=None, joint_equal=None,
             time_tsfm=None, scale_tsfm=None, action=None, save_path=None):
        assert eval_frame is not None
        dev = self.device
        sums = torch.zeros(len(eval_frame), dtype=torch.float32, device=dev)
        N = 0
        save_results = [] if save_path is not None else None
        index_cache = {}
        rank, world = _world()
        presharded = isinstance(getattr(test_loader, "sampler", None), torch.utils.data.DistributedSampler)
        # a presharded loader interleaves samples over the ranks (and pads with
        # duplicates): the saved results are put back in dataset order by the
        # sampler's per-sample indices
        sample_idx = np.asarray(list(iter(test_loader.sampler))) if presharded and save_path is not None else None
        # ... and its padding duplicates are the last of each rank's samples
        # (positions >= len(dataset) of the padded, interleaved index list):
        # the metric counts every dataset sample once, as a single process does
        n_real = self._presharded_real(test_loader.sampler) if presharded else None
        seen = 0
        self.model.eval()
        with torch.no_grad():
            for i, (inputs, _, _, all_seqs) in enumerate(test_loader):
                if world > 1 and not presharded and i % world != rank:
                    continue  # round-robin batch sharding over the ranks
                inputs = _to_dev(inputs, dev)
                all_seqs = all_seqs.float().to(dev, non_blocking=True).contiguous()
                outputs = self.inverse(self.model(self.transform(inputs), False))
                if isinstance(outputs, list):
                    outputs = outputs[0]
                    n, t = outputs.shape[:2]
                    outputs = outputs.view(n, t, -1)
                if scale_tsfm is not None:
                    outputs = scale_tsfm.inverse(outputs)
                if time_tsfm is not None:
                    outputs = time_tsfm.inverse(outputs)
                outputs = outputs.contiguous()
                n, seq_len, D = all_seqs.shape
                t_out0 = input_n if outputs.shape[1] != seq_len else 0
                key = (D, seq_len, t_out0)
                if key not in index_cache:
                    index_cache[key] = self._metric_indices(D, outputs.shape[2], seq_len, input_n, eval_frame,
                                                            dim_used, joint_to_ignore, joint_equal)
                used_pos, joint_src, frames = index_cache[key]
                k = n if n_real is None else min(n, max(0, n_real - seen))
                if k == n:
                    self._frame_metric(all_seqs, outputs, t_out0, used_pos, joint_src, frames, sums)
                elif k > 0:
                    self._frame_metric(all_seqs[:k].contiguous(), outputs[:k].contiguous(), t_out0, used_pos,
                                       joint_src, frames, sums)
                N += k
                if save_results is not None:
                    pred = self._fill_pred(all_seqs, outputs, used_pos, joint_src, t_out0)[:, input_n:]
                    targ = all_seqs.view(n, seq_len, -1, 3)[:, input_n:]
                    idx = sample_idx[seen:seen + n] if sample_idx is not None else None
                    save_results.append((i, rank, pred.cpu().numpy(), targ.cpu().numpy(), idx))
                seen += n
            if action is None:
                action = "NA"
            if world > 1:  # per-frame sums and sample counts of every rank
                from dstd_dist import reduce_partials
                sums, n_all = reduce_partials(sums, torch.tensor([float(N)], dtype=torch.float64, device=sums.device))
                N = float(n_all[0])
            t_metric = sums.double().cpu().numpy() / N  # the one synchronisation
            self.logger.info(f"action: {action}|test|loss:{t_metric.mean():.2f}")
            if save_results is not None:
                self._save_results(save_path, save_results, rank, world)
        # t_l.avg of the reference = sum over (batch, frame) of metric_k / (N * frames)
        return float(t_metric.mean()), t_metric

    @staticmethod
    def _presharded_real(sampler):
        """How many of this rank's samples from a DistributedSampler are
        dataset samples rather than padding: the rank reads positions
        rank, rank + world, ... of the index list padded to total_size, and
        the positions past len(dataset) are the duplicates."""
        n_data = len(sampler.dataset)
        if getattr(sampler, "drop_last", False) or sampler.total_size <= n_data:
            return sampler.num_samples
        r, w = sampler.rank, sampler.num_replicas
        return max(0, -(-(n_data - r) // w))

    @staticmethod
    def _save_results(save_path, parts, rank, world):
        """np.savez of every batch's (result, target) (:405-409).  With several
        ranks the per-rank parts are gathered to rank 0 and written by rank 0
        alone, in the single-process order: the engine's own round-robin batch
        sharding is undone by (batch index, rank); a presharded loader
        (DistributedSampler, samples interleaved over the ranks and padded with
        duplicates) by the sampler's per-sample dataset indices, each index
        kept once.  A rank without batches contributes nothing."""
        if world > 1:
            gathered = [None] * world
            dist.all_gather_object(gathered, parts)
            if rank != 0:
                return
            parts = sorted((p for g in gathered for p in g), key=lambda p: (p[0], p[1]))
        if not parts:
            return
        result = np.concatenate([p[2] for p in parts], 0)
        target = np.concatenate([p[3] for p in parts], 0)
        if parts[0][4] is not None:
            idx = np.concatenate([p[4] for p in parts], 0)
            _, first = np.unique(idx, return_index=True)  # sorted by dataset index, duplicates dropped
            result, target = result[first], target[first]
        np.savez(save_path + ".npz", target=target, result=result)

    def _frame_metric(self, all_seqs, outputs, t_out0, used_pos, joint_src, frames, sums):
        """sums[k] += sum over the batch of the MPJPE at frames[k] (:366-404),
        one kernel on the device (dstd_frame_mpjpe)."""
        n, seq_len, D = all_seqs.shape
        code = native.lib().dstd_frame_mpjpe(native.ptr(all_seqs, "all_seqs"), native.ptr(outputs, "outputs"), n,
                                             seq_len, D, t_out0, used_pos.data_ptr(), outputs.shape[2],
                                             joint_src.data_ptr(), frames.data_ptr(), len(frames), sums.data_ptr(),
                                             native.stream_handle(all_seqs.device))
        native.check(code, "dstd_frame_mpjpe")

    def _metric_indices(self, D, n_out_dims, seq_len, input_n, eval_frame, dim_used, joint_to_ignore, joint_equal):
        """Device index tables of the metric: used_pos[d] (position of dim d in
        the outputs or -1, :371-381), joint_src[j] (the ignore <- equal copy,
        :382-389) and the absolute eval frames (input_n + eval_frame[k])."""
        used_pos = np.full(D, -1, dtype=np.int32)
        if dim_used is None or np.any(np.asarray(dim_used, dtype=object) == None):  # noqa: E711
            used_pos[:] = np.arange(D)
        else:
            used_pos[np.asarray(dim_used, dtype=np.int64)] = np.arange(len(dim_used))
        if used_pos.max() + 1 != n_out_dims:
            raise ValueError(f"test: outputs have {n_out_dims} dims, dim_used selects {used_pos.max() + 1}")
        joint_src = np.arange(D // 3, dtype=np.int32)
        if joint_to_ignore is not None and not np.any(np.asarray(joint_to_ignore, dtype=object) == None):  # noqa
            assert joint_to_ignore.shape == joint_equal.shape
            joint_src[np.asarray(joint_to_ignore)] = np.asarray(joint_equal)
        frames = np.asarray([input_n + f for f in eval_frame], dtype=np.int32)
        if frames.max() >= seq_len:
            raise ValueError(f"eval frame {frames.max()} outside the {seq_len}-frame sequence")
        dev = self.device
        return (torch.from_numpy(used_pos).to(dev), torch.from_numpy(joint_src).to(dev),
                torch.from_numpy(frames).to(dev))

    @staticmethod
    def _fill_pred(all_seqs, outputs, used_pos, joint_src, t_out0):
        """pred_3d of :369-389 as a tensor (only for save_path)."""
        n, T, D = all_seqs.shape
        pred = all_seqs.clone()
        up = used_pos.long()
        sel = torch.nonzero(up >= 0).squeeze(1)
        pred[:, t_out0:, sel] = outputs[:, :, up[sel]]
        J = D // 3
        src = (joint_src.long()[:, None] * 3 + torch.arange(3, device=pred.device)[None]).reshape(-1)
        return pred[:, :, src].view(n, T, J, 3)


__all__ = ["ModelWrapper", "PredictionEngine", "AccumLoss"]
