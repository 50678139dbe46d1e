"""Race / memory-error detection on the native runtime (the reference runs
`go test -race`, .github/workflows/ci.yml:60-63): the lease queue and the
scheduler stress test built with ThreadSanitizer and with ASan+UBSan."""
import os

import pytest

from llm_mcp_amd.build import sanitize_runtime


@pytest.mark.skipif(not os.path.exists("/opt/rocm/llvm/bin/clang++")
                    and "LMX_SAN_CXX" not in os.environ, reason="no clang for sanitizers")
def test_runtime_under_tsan_and_asan():
    logs = sanitize_runtime()
    for name, log in logs.items():
        assert "queue:" in log and "scheduler:" in log and log.rstrip().endswith("ok"), name
