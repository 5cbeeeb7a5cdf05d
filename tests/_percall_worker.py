"""Worker of test_gpu_percall_service.py::test_staging_variants: per-message
calls (back-to-back and with gaps) against the oracle under the staging
variant the environment selects (CAPNP_PERCALL_BAR, CAPNP_SVC_LINE_BAR are
read once per process).  Exit status 0 when every call matched."""
import os
import sys
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_ROOT, os.path.join(_ROOT, "tests"), os.path.join(_ROOT, "capnproto-rust_amd"),
           os.path.join(_ROOT, "oracle")):
    sys.path.insert(0, _p)

import test_gpu_percall_service as T  # noqa: E402


def main():
    from capnp_amd import Context
    ctx = Context(0)
    try:
        for k, (segs, ref) in enumerate(T._messages(int(sys.argv[1]), 120)):
            assert T._write(ctx, segs) == ref, k
            T._read_check(ctx, ref, k)
            if k % 10 == 9:
                time.sleep(0.002)  # (past the warm window: a one-shot launch)
    finally:
        ctx.close()
    print("ok")


if __name__ == "__main__":
    main()
