"""Learning-rate schedule, the train-loss metric and the early-stop checkpoint
saver (reference: utils/utils.py:35-50, 120-154; tf.keras.metrics.Mean as used
at utils/pipeline.py:35,80 and train.py:47,56).

CustomSchedule is evaluated on the device inside fpnmt_amsgrad_step (from the
device-resident `iterations` counter); this host object carries its constants
and gives the same value for inspection / tests.
"""
import numpy as np
import torch

from common.common_definitions import EPOCHS, GAP_OF_DEAD_EPOCH, MIN_EPOCH_TO_BREAK


class CustomSchedule:
    def __init__(self, d_model, warmup_steps=4000, multiplier=1):
        self.d_model = float(d_model)
        self.warmup_steps = warmup_steps
        self.multiplier = multiplier

    def __call__(self, step):
        """fp32 arithmetic like the reference's tf ops; lr(0) = 0."""
        f = np.float32
        step = f(step)
        with np.errstate(divide="ignore"):
            rs = f(1.0) / np.sqrt(step) if step > 0 else f(np.inf)
        arg1 = rs / np.maximum((step - f(self.warmup_steps)) * f(self.multiplier) / f(self.warmup_steps * 2), f(1))
        arg2 = step * f(self.warmup_steps ** -1.5)
        return float(f(1.0) / np.sqrt(f(self.d_model)) * np.minimum(arg1, arg2))


class Mean:
    """tf.keras.metrics.Mean(name): running mean of the values passed to
    __call__ (each with weight 1). The running total and count stay on the
    device of the first value, so updating it inside the training loop never
    synchronises with the host; result() copies the scalar out (as a 0-d CPU
    tensor, so ``result().numpy()`` works like the Keras metric's)."""

    def __init__(self, name="mean"):
        self.name = name
        self._total = None
        self._count = None

    def __call__(self, value):
        v = torch.as_tensor(value).detach().to(torch.float32).reshape(-1)
        if self._total is None or self._total.device != v.device:
            self._total = torch.zeros((), dtype=torch.float32, device=v.device)
            self._count = torch.zeros((), dtype=torch.float32, device=v.device)
        self._total.add_(v.sum())
        self._count.add_(float(v.numel()))
        return self.result_tensor()

    update_state = __call__

    def reset_states(self):
        if self._total is not None:
            self._total.zero_()
            self._count.zero_()

    reset_state = reset_states

    def result_tensor(self):
        """The mean as a device scalar (0 before the first update, as Keras'
        divide_no_nan)."""
        if self._total is None:
            return torch.zeros((), dtype=torch.float32)
        return torch.where(self._count > 0, self._total / self._count.clamp_min(1.0), self._total.new_zeros(()))

    def result(self):
        return self.result_tensor().cpu()


class SmartCheckpointSaver:
    """Early-stopping checkpoint policy of utils/utils.py:120-154: save when
    the validation score improves; after MIN_EPOCH_TO_BREAK epochs, return -1
    once min(EPOCHS, max(MIN_EPOCH_TO_BREAK, 2*best_epoch), best_epoch +
    GAP_OF_DEAD_EPOCH) epochs have passed without improvement.

    Returns 1 (checkpoint saved), 0 (nothing done) or -1 (stop training)."""

    def __init__(self, ckpt_manager, epochs=EPOCHS, min_epoch_to_break=MIN_EPOCH_TO_BREAK,
                 gap_of_dead_epoch=GAP_OF_DEAD_EPOCH):
        self.ckpt_manager = ckpt_manager
        self.max_val_acc = -np.inf
        self.max_acc_epoch = 0
        self.epochs = epochs
        self.min_epoch_to_break = min_epoch_to_break
        self.gap_of_dead_epoch = gap_of_dead_epoch

    def __call__(self, curr_epoch, curr_val_acc):
        if self.max_acc_epoch == 0:  # first evaluation (utils.py:135-137)
            self.max_val_acc = curr_val_acc
            self.max_acc_epoch = curr_epoch
        if curr_val_acc > self.max_val_acc:
            path = self.ckpt_manager.save()
            print("Saving checkpoint for epoch {} at {}".format(curr_epoch, path))
            self.max_val_acc = curr_val_acc
            self.max_acc_epoch = curr_epoch
            return 1
        elif curr_epoch <= self.min_epoch_to_break:
            self.max_val_acc = curr_val_acc
            self.max_acc_epoch = curr_epoch
        else:
            epoch_min = min(self.epochs, max(self.min_epoch_to_break, int(self.max_acc_epoch * 2.)),
                            int(self.max_acc_epoch + self.gap_of_dead_epoch))
            if epoch_min <= curr_epoch:
                return -1
        return 0
