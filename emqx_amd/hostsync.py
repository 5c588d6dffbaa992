"""Host-side barrier and max-reduce for one-process-per-GPU runs on one node.

Replicated mode (BASELINE config C3) has no data-path collective, so the ranks
only need to line up around the timed region and agree on the slowest rank's
time.  That is done through files in a per-run directory, not through
torch.distributed: loading torch's bundled HIP runtime into a process whose
engine already runs on /opt/rocm's makes torch's GPU init fail,
and a process that never touches torch keeps exactly one HIP runtime.

The run key is the launcher's pid (torchrun's agent is every rank's parent)
plus MASTER_PORT, so concurrent or stale runs never share a directory.
"""

from __future__ import annotations

import os
import time


class FileGroup:
    def __init__(self, rank: int, world: int, key: str = None, root: str = "/tmp"):
        self.rank, self.world = rank, world
        key = key or f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"
        self.dir = os.path.join(root, f"emqx_tm_sync_{key}")
        os.makedirs(self.dir, exist_ok=True)
        self._n = 0

    def _post(self, tag: str, payload: str):
        tmp = os.path.join(self.dir, f".{tag}.{self.rank}.tmp")
        with open(tmp, "w") as f:
            f.write(payload)
        os.replace(tmp, os.path.join(self.dir, f"{tag}.{self.rank}"))   # atomic publish

    def _collect(self, tag: str, timeout: float):
        paths = [os.path.join(self.dir, f"{tag}.{r}") for r in range(self.world)]
        t0 = time.monotonic()
        nap = 20e-6
        while not all(os.path.exists(p) for p in paths):
            waited = time.monotonic() - t0
            if waited > timeout:
                raise TimeoutError(f"rank {self.rank}: barrier {tag} timed out")
            # short naps while the ranks are close (the barriers around the
            # timed region), then backing off: ranks waiting out rank 0's CPU
            # baseline must not take the cores it is timing
            if waited > 0.05:
                nap = min(nap * 2, 2e-3)
            time.sleep(nap)
        out = []
        for p in paths:
            with open(p) as f:
                out.append(f.read())
        return out

    def barrier(self, timeout: float = 600.0):
        self._n += 1
        tag = f"b{self._n}"
        self._post(tag, "")
        self._collect(tag, timeout)

    def allmax(self, value: float, timeout: float = 600.0) -> float:
        self._n += 1
        tag = f"m{self._n}"
        self._post(tag, repr(float(value)))
        return max(float(v) for v in self._collect(tag, timeout))

    def allgather(self, payload: str, timeout: float = 600.0) -> list:
        """Every rank's payload (a string), in rank order."""
        self._n += 1
        tag = f"g{self._n}"
        self._post(tag, payload)
        return self._collect(tag, timeout)

    def close(self):
        """Every rank reports it is done reading; then rank 0 removes the directory."""
        self._post("done", "")
        if self.rank == 0:
            self._collect("done", 600.0)
            for name in os.listdir(self.dir):
                try:
                    os.remove(os.path.join(self.dir, name))
                except OSError:
                    pass
            try:
                os.rmdir(self.dir)
            except OSError:
                pass
