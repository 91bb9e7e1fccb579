"""Learning-rate schedule (reference: utils/utils.py:35-50).

CustomSchedule is evaluated on the device inside fpnmt_amsgrad_step (from the
device-resident `iterations` counter); this host object carries its constants
and gives the same value for inspection / tests.
"""
import math

import numpy as np


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
