"""Training/evaluation engine with the reference ``train_utils`` surface.

Restates ``train_utils/train_and_eval.py`` (and re-exports the criterion of
``stfunet.loss``) so a ``train.py``-style driver can import from here:

* ``preprocess_input``      :9-22   (flat_channels / average_frame / time_sequence)
* ``ConfusionMatrix``       :25-70
* ``DiceCoefficient``       :73-142 -- ``reduce_from_all_processes`` all-reduces a
  *tensor* count (the reference passes a Python int to ``all_reduce``, :132,
  which raises under any process group; SURVEY.md section 0, defect 2)
* ``SmoothedValue``/``MetricLogger`` :145-296 (same printed format)
* ``criterion``             :299-313 (gfx950 kernels, ``stfunet.loss``)
* ``evaluate``              :316-374
* ``train_one_epoch``       :377-411 (autocast when a GradScaler is given,
  zero_grad -> backward -> step -> per-iteration LR step -> ``loss.item()``)
* ``create_lr_scheduler``   :414-438

and the per-epoch artefacts of ``train.py``'s loop: ``results_file_name`` /
``write_epoch_results`` (train.py:155-162, 289-301), ``print_eval`` (:278-284),
``checkpoint_dict`` (:304-311, ``scaler`` key under ``--amp``), ``resume_from``
(:249-256) and ``EarlyStopping`` (train_utils/early_stopping.py:9-24).
"""
import datetime
import os
import time
from collections import defaultdict, deque

import numpy as np
import torch
import torch.distributed as dist

from .loss import criterion  # noqa: F401  (re-export, reference name)


def preprocess_input(inputs, model):
    fmt = getattr(model, "input_format", "time_sequence")
    if fmt == "flat_channels":
        b, t, c, h, w = inputs.shape
        return inputs.view(b, t * c, h, w)
    if fmt == "average_frame":
        return inputs.mean(dim=1)
    if fmt == "time_sequence":
        return inputs
    raise ValueError(f"Unsupported input_format: {fmt}")


def _dist_on():
    return dist.is_available() and dist.is_initialized()


class ConfusionMatrix:
    """rows = target class, columns = predicted class (train_and_eval.py:30-39)."""

    def __init__(self, num_classes):
        self.num_classes = num_classes
        self.mat = None

    def update(self, a, b):
        n = self.num_classes
        if self.mat is None:
            self.mat = torch.zeros((n, n), dtype=torch.int64, device=a.device)
        with torch.no_grad():
            keep = (a >= 0) & (a < n)
            self.mat += torch.bincount(n * a[keep].to(torch.int64) + b[keep], minlength=n * n).reshape(n, n)

    def reset(self):
        self.mat.zero_()

    def compute(self):
        h = self.mat.float()
        diag = torch.diag(h)
        return diag.sum() / h.sum(), diag / h.sum(1), diag / (h.sum(1) + h.sum(0) - diag)

    def reduce_from_all_processes(self):
        if not _dist_on():
            return
        dist.barrier()
        dist.all_reduce(self.mat)

    def __str__(self):
        acc_global, acc, iu = self.compute()
        return ("global correct: {:.1f}\naverage row correct: {}\nIoU: {}\nmean IoU: {:.1f}").format(
            acc_global.item() * 100, ["{:.1f}".format(i) for i in (acc * 100).tolist()],
            ["{:.1f}".format(i) for i in (iu * 100).tolist()], iu.mean().item() * 100)


class DiceCoefficient:
    """Per-batch Dice of argmax predictions, averaged over batches (:80-138)."""

    def __init__(self, num_classes=2, ignore_index=None):
        self.num_classes = num_classes
        self.ignore_index = ignore_index
        self.cumulative_dice = None
        self.count = None

    def update(self, pred, target):
        if isinstance(pred, dict):
            pred = pred["out"]
        # softmax first, as the reference does (:84-85): fp32 softmax can round two logits that
        # differ by less than an ulp of exp() to the same probability, and argmax then takes the
        # first of the tie where argmax(x) would not
        pred = torch.argmax(torch.softmax(pred, dim=1), dim=1)
        if self.ignore_index is not None:
            keep = target != self.ignore_index
            pred = pred * keep
            target = target * keep
        pred = pred.reshape(-1)
        target = target.reshape(-1)
        per = []
        for c in range(self.num_classes):
            pc = pred == c
            tc = target == c
            union = pc.sum() + tc.sum()
            inter = (pc & tc).sum()
            per.append(torch.where(union > 0, 2.0 * inter.float() / union.clamp_min(1).float(),
                                   torch.ones((), device=pred.device)))
        d = torch.stack(per)
        if self.cumulative_dice is None:
            self.cumulative_dice = d
            self.count = 1
        else:
            self.cumulative_dice = self.cumulative_dice + d
            self.count += 1

    def compute(self):
        if not self.count:
            return torch.tensor(0.0)
        return self.cumulative_dice / self.count

    def reduce_from_all_processes(self):
        if not _dist_on() or self.cumulative_dice is None:
            return
        dist.barrier()
        dist.all_reduce(self.cumulative_dice)
        cnt = torch.tensor([float(self.count)], dtype=torch.float64, device=self.cumulative_dice.device)
        dist.all_reduce(cnt)
        self.count = int(round(cnt.item()))

    @property
    def value(self):
        if self.cumulative_dice is None:
            return torch.tensor(0.0)
        return self.compute().mean()

    def reset(self):
        self.cumulative_dice = None
        self.count = 0


class SmoothedValue:
    def __init__(self, window_size=20, fmt=None):
        self.deque = deque(maxlen=window_size)
        self.total = 0.0
        self.count = 0
        self.fmt = fmt or "{median:.4f} ({global_avg:.4f})"

    def update(self, value, n=1):
        self.deque.append(value)
        self.count += n
        self.total += value * n

    def synchronize_between_processes(self):
        if not _dist_on():
            return
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        t = torch.tensor([self.count, self.total], dtype=torch.float64, device=dev)
        dist.barrier()
        dist.all_reduce(t)
        self.count, self.total = int(t[0].item()), t[1].item()

    @property
    def median(self):
        return torch.tensor(list(self.deque)).median().item()

    @property
    def avg(self):
        return torch.tensor(list(self.deque), dtype=torch.float32).mean().item()

    @property
    def global_avg(self):
        return self.total / self.count if self.count > 0 else 0

    @property
    def max(self):
        return max(self.deque)

    @property
    def value(self):
        return self.deque[-1]

    def __str__(self):
        return self.fmt.format(median=self.median, avg=self.avg, global_avg=self.global_avg, max=self.max,
                               value=self.value)


class MetricLogger:
    def __init__(self, delimiter="\t"):
        self.meters = defaultdict(SmoothedValue)
        self.delimiter = delimiter

    def update(self, **kwargs):
        for k, v in kwargs.items():
            if isinstance(v, torch.Tensor):
                v = v.item()
            assert isinstance(v, (float, int))
            self.meters[k].update(v)

    def __getattr__(self, attr):
        meters = self.__dict__.get("meters", {})
        if attr in meters:
            return meters[attr]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{attr}'")

    def __str__(self):
        return self.delimiter.join(f"{name}: {meter}" for name, meter in self.meters.items())

    def synchronize_between_processes(self):
        for meter in self.meters.values():
            meter.synchronize_between_processes()

    def add_meter(self, name, meter):
        self.meters[name] = meter

    def log_every(self, iterable, print_freq, header=None):
        header = header or ""
        start = end = time.time()
        iter_time = SmoothedValue(fmt="{avg:.4f}")
        data_time = SmoothedValue(fmt="{avg:.4f}")
        n = len(iterable)
        width = len(str(n))
        parts = [header, "[{0:" + str(width) + "d}/{1}]", "eta: {eta}", "{meters}", "time: {time}", "data: {data}"]
        if torch.cuda.is_available():
            parts.append("max mem: {memory:.0f}")
        msg = self.delimiter.join(parts)
        for i, obj in enumerate(iterable):
            data_time.update(time.time() - end)
            yield obj
            iter_time.update(time.time() - end)
            if i % print_freq == 0 or i == n - 1:
                eta = str(datetime.timedelta(seconds=int(iter_time.global_avg * (n - i))))
                kw = dict(eta=eta, meters=str(self), time=str(iter_time), data=str(data_time))
                if torch.cuda.is_available():
                    kw["memory"] = torch.cuda.max_memory_allocated() / (1024.0 * 1024.0)
                print(msg.format(i, n, **kw))
            end = time.time()
        total = time.time() - start
        print("{} Total time: {} ({:.4f} s / it)".format(header, str(datetime.timedelta(seconds=int(total))),
                                                         total / max(n, 1)))


def eval_update(out, target, confmat, dice):
    """One batch of evaluate(): ``confmat.update(target, output.argmax(1))`` +
    ``dice.update(output, target)`` as ONE stf_eval_counts_sm pass (confusion counts from
    the logits' first argmax, per-class Dice counts from the first argmax of
    ``torch.softmax(output, 1)`` -- the very op DiceCoefficient.update runs, :84-85, so
    near-ties round the same way; no host synchronisation), then the per-batch Dice from
    the counts exactly as DiceCoefficient.update computes it (train_and_eval.py:80-118)."""
    from ._lib import call, stream
    from .nhwc import _p
    if not out.is_cuda:
        raise RuntimeError("engine.evaluate runs the gfx950 stf_eval_counts kernel: logits must be on a ROCm "
                           "device (no CPU fallback)")
    out = out.detach().float().contiguous()
    target = target.to(device=out.device, dtype=torch.int64).contiguous()
    B, K = out.shape[:2]
    if confmat.mat is None:
        confmat.mat = torch.zeros((K, K), dtype=torch.int64, device=out.device)
    counts = torch.zeros((K, 3), dtype=torch.int64, device=out.device)
    ign = dice.ignore_index if dice.ignore_index is not None else -1
    probs = torch.softmax(out, dim=1)
    call("stf_eval_counts_sm", _p(out), _p(probs), _p(target), B, K, out[0, 0].numel(), ign, _p(confmat.mat),
         _p(counts), stream())
    inter, psum, tsum = counts.float().unbind(1)
    union = psum + tsum
    d = torch.where(union > 0, 2.0 * inter / union.clamp_min(1.0), torch.ones_like(union))
    if dice.cumulative_dice is None:
        dice.cumulative_dice = d
        dice.count = 1
    else:
        dice.cumulative_dice = dice.cumulative_dice + d
        dice.count += 1


def evaluate(model, data_loader, device, num_classes):
    model.eval()
    confmat = ConfusionMatrix(num_classes)
    dice = DiceCoefficient(num_classes=num_classes, ignore_index=255)
    logger = MetricLogger(delimiter="  ")
    with torch.no_grad():
        for image, target in logger.log_every(data_loader, 100, "Test:"):
            image = preprocess_input(image, model).to(device)
            target = target.to(device)
            out = model(image)["out"]
            eval_update(out, target, confmat, dice)
        confmat.reduce_from_all_processes()
        dice.reduce_from_all_processes()
        mat = confmat.mat.cpu().numpy()
    eps = 1e-6
    total = mat.sum()
    global_accuracy = np.diag(mat).sum() / total if total != 0 else 0.0
    class_metrics = []
    for c in range(num_classes):
        tp = mat[c, c]
        fp = mat[:, c].sum() - tp
        fn = mat[c, :].sum() - tp
        class_metrics.append({"precision": tp / (tp + fp + eps), "recall": tp / (tp + fn + eps),
                              "iou": tp / (tp + fp + fn + eps)})
    mean_metrics = {k2: np.mean([m[k1] for m in class_metrics])
                    for k1, k2 in (("precision", "mprecision"), ("recall", "mrecall"), ("iou", "miou"))}
    return {"dice": dice.value.item(), "confusion_matrix": confmat, "global_accuracy": global_accuracy,
            "class_metrics": class_metrics, "mean_metrics": mean_metrics}


def train_one_epoch(model, optimizer, data_loader, device, epoch, num_classes, lr_scheduler=None,
                    print_freq=10, scaler=None):
    model.train()
    logger = MetricLogger(delimiter="  ")
    logger.add_meter("lr", SmoothedValue(window_size=1, fmt="{value:.6f}"))
    lr = optimizer.param_groups[0]["lr"]
    for image, target in logger.log_every(data_loader, print_freq, f"Epoch: [{epoch}]"):
        image = preprocess_input(image, model).to(device)
        target = target.to(device)
        with torch.amp.autocast(device_type="cuda", enabled=scaler is not None):
            loss = criterion(model(image), target)
        optimizer.zero_grad()
        if scaler is not None:
            scaler.scale(loss).backward()
            scaler.step(optimizer)
            scaler.update()
        else:
            loss.backward()
            optimizer.step()
        lr_scheduler.step()
        lr = optimizer.param_groups[0]["lr"]
        logger.update(loss=loss.item(), lr=lr)
    # the epoch's last steps: a device-side failure flag (cooperative LSTM hand-off timeout)
    # raises here instead of at the next epoch's first step
    # (through a DistributedDataParallel-style wrapper's .module as well)
    prog = getattr(getattr(model, "module", model), "_program", None)
    if prog is not None and hasattr(prog, "check_device_errors"):
        prog.check_device_errors(block=True)
    return logger.meters["loss"].global_avg, lr


def lr_lambda(num_step, epochs, warmup=True, warmup_epochs=1, warmup_factor=1e-3):
    """Factor of create_lr_scheduler: linear warm-up, then poly(0.9) decay."""
    if not warmup:
        warmup_epochs = 0
    w = warmup_epochs * num_step

    def f(x):
        if warmup and x <= w:
            a = float(x) / w
            return warmup_factor * (1 - a) + a
        return (1 - (x - w) / ((epochs - warmup_epochs) * num_step)) ** 0.9
    return f


def create_lr_scheduler(optimizer, num_step: int, epochs: int, warmup=True, warmup_epochs=1, warmup_factor=1e-3):
    assert num_step > 0 and epochs > 0
    return torch.optim.lr_scheduler.LambdaLR(
        optimizer, lr_lambda=lr_lambda(num_step, epochs, warmup, warmup_epochs, warmup_factor))


# ---------------------------------------------------------------- train.py's epoch artefacts
def results_file_name(model_name, use_pk_maps=False, now=None, out_dir="./output"):
    """``./output/{model}_results_{MMDD-HHMM}{_pk}.txt`` (train.py:151-162); creates the
    directory like the reference."""
    now = now or datetime.datetime.now()
    os.makedirs(out_dir, exist_ok=True)
    return os.path.join(out_dir, "{}_results_{}{}.txt".format(model_name, now.strftime("%m%d-%H%M"),
                                                            "_pk" if use_pk_maps else ""))


def epoch_results_text(epoch, mean_loss, lr, eval_metrics):
    """The block train.py:289-301 appends to the results file after every epoch."""
    mm = eval_metrics["mean_metrics"]
    return (f"[epoch: {epoch}]\n"
            f"train_loss: {mean_loss:.4f}\n"
            f"lr: {lr:.6f}\n"
            f"dice: {eval_metrics['dice']:.4f}\n"
            f"global_acc: {eval_metrics['global_accuracy']:.4f}\n"
            f"mean_iou: {mm['miou']:.4f}\n"
            f"mean_precision: {mm['mprecision']:.4f}\n"
            f"mean_recall: {mm['mrecall']:.4f}\n"
            f"{eval_metrics['confusion_matrix']}\n\n")


def write_epoch_results(results_file, epoch, mean_loss, lr, eval_metrics):
    if results_file:
        with open(results_file, "a") as f:
            f.write(epoch_results_text(epoch, mean_loss, lr, eval_metrics))


def print_eval(eval_metrics):
    """The validation printout of train.py:278-284."""
    mm = eval_metrics["mean_metrics"]
    print(eval_metrics["confusion_matrix"])
    print(f"Dice coefficient: {eval_metrics['dice']:.4f}")
    print(f"Global accuracy: {eval_metrics['global_accuracy']:.4f}")
    print(f"Mean IoU: {mm['miou']:.4f}")
    print(f"Mean precision: {mm['mprecision']:.4f}")
    print(f"Mean recall: {mm['mrecall']:.4f}")


def checkpoint_dict(model, optimizer, lr_scheduler, epoch, args, scaler=None):
    """train.py:304-311: {'model', 'optimizer', 'lr_scheduler', 'epoch', 'args'} plus
    'scaler' when training with --amp (a GradScaler)."""
    save = {"model": model.state_dict(), "optimizer": optimizer.state_dict(),
            "lr_scheduler": lr_scheduler.state_dict(), "epoch": epoch, "args": args}
    if scaler is not None:
        save["scaler"] = scaler.state_dict()
    return save


def resume_from(checkpoint, model, optimizer, lr_scheduler, scaler=None):
    """train.py:249-256: load model / optimizer / scheduler (and the GradScaler under
    --amp) and return the next epoch."""
    model.load_state_dict(checkpoint["model"])
    optimizer.load_state_dict(checkpoint["optimizer"])
    lr_scheduler.load_state_dict(checkpoint["lr_scheduler"])
    if scaler is not None and "scaler" in checkpoint:
        scaler.load_state_dict(checkpoint["scaler"])
    return checkpoint["epoch"] + 1


class EarlyStopping:
    """train_utils/early_stopping.py:9-24 (patience on a higher-is-better metric)."""

    def __init__(self, patience=10, verbose=False):
        self.patience = patience
        self.counter = 0
        self.best_score = None
        self.early_stop = False
        self.verbose = verbose

    def step(self, metric):
        if self.best_score is None:
            self.best_score = metric
            return False
        if metric <= self.best_score:
            self.counter += 1
            if self.verbose:
                print(f"EarlyStopping: {self.counter}/{self.patience} no improvement.")
            if self.counter >= self.patience:
                self.early_stop = True
                return True
        else:
            self.best_score = metric
            self.counter = 0
        return False
