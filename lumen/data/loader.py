"""Background batch preparation: indexing, tokenised-row fetch and collation run on a host
thread, ``depth`` batches ahead of the training loop, into pinned memory.

The reference's HF Trainer builds each batch synchronously in the step loop (DataLoader with
num_workers=0, training/train_baseline.py:200-205); here the step loop only issues the
non-blocking host-to-device copies of a batch that is already collated and pinned, so host-side
data work overlaps the GPU step instead of sitting between steps.
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Dict, Iterable, Iterator, Optional

import torch

_END = object()


def pin_batch(b: Dict) -> Dict:
    if not torch.cuda.is_available():
        return b
    return {k: (v.pin_memory() if isinstance(v, torch.Tensor) else v) for k, v in b.items()}


class PrefetchLoader:
    """Iterate ``collate(raw)`` for raw batches of ``source`` on a daemon thread.

    Yields ``(raw, batch)``; exceptions raised by the producer are re-raised in the consumer.
    ``close()`` (or exhausting the iterator) stops the thread."""

    def __init__(self, source: Iterable, collate: Callable, depth: int = 2, pin: bool = True):
        self._src = iter(source)
        self._collate = collate
        self._q: "queue.Queue" = queue.Queue(maxsize=max(1, depth))
        self._stop = threading.Event()
        self._pin = pin
        self._t = threading.Thread(target=self._run, name="lumen-prefetch", daemon=True)
        self._t.start()

    def _run(self):
        try:
            for raw in self._src:
                if self._stop.is_set():
                    return
                b = self._collate(raw)
                if self._pin:
                    b = pin_batch(b)
                while not self._stop.is_set():
                    try:
                        self._q.put((raw, b), timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:  # noqa: BLE001 - handed to the consumer
            self._q.put(e)
            return
        self._q.put(_END)

    def __iter__(self) -> Iterator:
        while True:
            item = self._q.get()
            if item is _END:
                return
            if isinstance(item, BaseException):
                raise item
            yield item

    def close(self, timeout: Optional[float] = 5.0):
        self._stop.set()
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass
        self._t.join(timeout)
