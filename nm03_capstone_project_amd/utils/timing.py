import time


class Timer:
    """Wall-clock context manager: `with Timer() as t: ...; t.elapsed`."""

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.elapsed = time.perf_counter() - self.t0
        return False
