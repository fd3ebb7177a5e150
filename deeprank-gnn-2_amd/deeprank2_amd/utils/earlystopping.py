"""Early-stopping trigger for ``Trainer.train`` (drop-in for
``deeprank2.utils.earlystopping.EarlyStopping``; behaviour pinned by the
reference's ``tests/utils/test_earlystopping.py`` cases, restated in
``tests/test_trainer.py``).

Two independent triggers, evaluated once per epoch:

* stall: an epoch whose validation loss is above ``best - delta`` is a
  stalled epoch (equal counts as progress); ``patience`` stalled epochs in a row stop training.  A
  non-stalled epoch resets the run.  ``best`` is the lowest validation loss
  seen so far (it also moves down on a stalled epoch whose loss is below it
  by less than ``delta``).
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
        self.val_loss_min = None  # lowest validation loss so far

    @property
    def best_score(self):
        """The reference keeps the negated best loss under this name."""
        return None if self.val_loss_min is None else -self.val_loss_min

    def _stalled(self, val_loss: float) -> bool:
        return val_loss > self.val_loss_min - self.delta

    def __call__(self, epoch: int, val_loss: float, train_loss: float | None = None):
        first = self.val_loss_min is None
        if not first:
            previous = self.val_loss_min
            if self._stalled(val_loss):
                self.counter += 1
                if self.verbose:
                    margin = f"by more than {self.delta} " if self.delta else ""
                    self.trace_func(f"Validation loss did not decrease {margin}({previous:.6f} --> {val_loss:.6f}); stalled epochs: {self.counter} of {self.patience}")
                if self.counter >= self.patience:
                    self.trace_func(f"EarlyStopping activated at epoch # {epoch}: no improvement for {self.patience} epochs (patience reached).")
                    self.early_stop = True
            else:
                self.counter = 0
                if self.verbose:
                    self.trace_func(f"Validation loss decreased ({previous:.6f} --> {val_loss:.6f}).")
        if first or val_loss <= self.val_loss_min:
            self.val_loss_min = val_loss
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
