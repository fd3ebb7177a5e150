"""Early-stopping trigger for ``Trainer.train`` (drop-in for
``deeprank2.utils.earlystopping.EarlyStopping``; behaviour pinned by the
reference's ``tests/utils/test_earlystopping.py`` cases, restated in
``tests/test_trainer.py``).

Two independent triggers, evaluated once per epoch:

* stall: an epoch whose validation loss is above ``best - delta`` is a
  stalled epoch (equal counts as progress); ``patience`` stalled epochs in a
  row stop training.  A non-stalled epoch resets the run.  ``best`` is the
  lowest validation loss seen so far (it also moves down on a stalled epoch
  whose loss is below it by less than ``delta``); a NaN validation loss
  resets the run and makes the next epoch count as progress, as in the
  reference.
* overfitting: after ``min_epoch``, a validation loss above the training loss
  by more than ``maxgap`` stops training at once.
"""

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
        self.counter = 0  # stalled epochs in the current run
        self.best_score = None  # the negated best validation loss (NaN after a NaN epoch, as the reference)
        self.val_loss_min = None  # the validation loss that set best_score

    def _stall(self, epoch, val_loss):
        self.counter += 1
        if self.verbose:
            margin = f"by more than {self.delta} " if self.delta else ""
            self.trace_func(f"Validation loss did not decrease {margin}({self.val_loss_min:.6f} --> {val_loss:.6f}); stalled epochs: {self.counter} of {self.patience}")
        if self.counter >= self.patience:
            self.trace_func(f"EarlyStopping activated at epoch # {epoch}: no improvement for {self.patience} epochs (patience reached).")
            self.early_stop = True

    def __call__(self, epoch: int, val_loss: float, train_loss: float | None = None):
        # The comparisons run on the negated loss exactly as the reference's
        # (earlystopping.py:47-70), so a NaN loss behaves the same: it is
        # never "stalled" (NaN < x is False), it resets the run and leaves
        # best_score NaN, and the next finite epoch then always counts as progress.
        score = -val_loss
        if self.best_score is None:
            self.best_score, self.val_loss_min = score, val_loss
        elif score < self.best_score + self.delta:
            self._stall(epoch, val_loss)
        else:
            if self.verbose:
                self.trace_func(f"Validation loss decreased ({self.val_loss_min:.6f} --> {val_loss:.6f}).")
            self.best_score, self.counter = score, 0
        if score >= self.best_score:
            self.best_score, self.val_loss_min = score, val_loss
        self._check_gap(epoch, val_loss, train_loss)

    def _check_gap(self, epoch, val_loss, train_loss):
        if not self.maxgap or epoch <= self.min_epoch:
            return
        if train_loss is None:
            msg = "Cannot compute gap because no train_loss is provided to EarlyStopping."
            raise ValueError(msg)
        gap = val_loss - train_loss
        if gap > self.maxgap:
            self.trace_func(f"EarlyStopping activated at epoch # {epoch}: overfitting, validation exceeds training loss by {gap} (maximum allowed {self.maxgap}).")
            self.early_stop = True
