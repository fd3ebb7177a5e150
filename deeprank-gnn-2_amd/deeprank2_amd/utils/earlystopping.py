"""Early stopping with the reference's trigger rules
(``deeprank2/utils/earlystopping.py``): stop after ``patience`` epochs without
a validation-loss improvement of more than ``delta``, or, past ``min_epoch``,
when validation loss exceeds training loss by more than ``maxgap``."""

from __future__ import annotations

from collections.abc import Callable


class EarlyStopping:
    def __init__(self, patience: int = 10, delta: float = 0, maxgap: float | None = None, min_epoch: int = 10, verbose: bool = True, trace_func: Callable = print):
        self.patience = patience
        self.delta = delta
        self.maxgap = maxgap
        self.min_epoch = min_epoch
        self.verbose = verbose
        self.trace_func = trace_func
        self.early_stop = False
        self.counter = 0
        self.best_score = None
        self.val_loss_min = None

    def __call__(self, epoch: int, val_loss: float, train_loss: float | None = None):
        score = -val_loss
        if self.best_score is None:
            self.best_score, self.val_loss_min = score, val_loss
        elif score < self.best_score + self.delta:
            self.counter += 1
            if self.verbose:
                self.trace_func(f"Validation loss did not decrease ({self.val_loss_min:.6f} --> {val_loss:.6f}). EarlyStopping counter: {self.counter} out of {self.patience}")
            if self.counter >= self.patience:
                self.trace_func(f"EarlyStopping activated at epoch # {epoch} because patience of {self.patience} has been reached.")
                self.early_stop = True
        else:
            if self.verbose:
                self.trace_func(f"Validation loss decreased ({self.val_loss_min:.6f} --> {val_loss:.6f}).")
            self.best_score = score
            self.counter = 0
        if score >= self.best_score:
            self.best_score, self.val_loss_min = score, val_loss
        if self.maxgap and epoch > self.min_epoch:
            if train_loss is None:
                msg = "Cannot compute gap because no train_loss is provided to EarlyStopping."
                raise ValueError(msg)
            gap = val_loss - train_loss
            if gap > self.maxgap:
                self.trace_func(f"EarlyStopping activated at epoch # {epoch} due to overfitting. The difference between validation and training loss of {gap} exceeds the maximum allowed ({self.maxgap})")
                self.early_stop = True
