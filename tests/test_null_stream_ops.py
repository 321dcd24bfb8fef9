"""CPU: no product source issues a memory operation on the null stream.

The host context once zeroed its arena with hipMemset, which runs on the null stream (torch's
default stream). Its non-blocking streams do not wait for that fill, so the fill could land
after the first call's uploads (profiles/r06/intermittent/README.md §6;
scripts/microbench/memset_race.hip shows the race). Every copy and fill now goes on a stream
the call orders itself. This test keeps it that way: the synchronous null-stream forms, and
the async forms given stream 0 / nullptr, are refused in fury_amd/csrc. The one exception is
the internal profiling counters' read-back (varlen.hip, g_prof), which runs after a device
sync and feeds no product path."""
import glob
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SYNC_FORMS = re.compile(r"\bhip(Memset|Memcpy|MemsetD8|MemsetD16|MemsetD32|MemcpyHtoD|MemcpyDtoH|MemcpyDtoD)\s*\(")
ASYNC_NULL = re.compile(r"\bhip(MemsetAsync|MemcpyAsync)\s*\((?:[^;]*),\s*(0|nullptr|NULL|hipStreamNull)\s*\)\s*[;)]")
ALLOWED = ("g_prof",)


def product_sources():
    files = []
    for pat in ("*.cpp", "*.hip", "*.h"):
        files += glob.glob(os.path.join(REPO, "fury_amd", "csrc", pat))
    assert files, "no product sources found"
    return sorted(files)


def test_no_null_stream_memory_ops():
    bad = []
    for path in product_sources():
        with open(path, encoding="utf-8") as fh:
            for no, line in enumerate(fh, 1):
                code = line.split("//", 1)[0]
                if any(a in code for a in ALLOWED):
                    continue
                if SYNC_FORMS.search(code) or ASYNC_NULL.search(code):
                    bad.append(f"{os.path.relpath(path, REPO)}:{no}: {line.strip()}")
    assert bad == [], "null-stream memory operations:\n" + "\n".join(bad)


def test_the_check_sees_the_round6_form():
    old = "  if (!rc) rc = hip_check(hipMemset(c->arena, 0, (size_t)(2 * per)), \"hipMemset(arena)\");"
    assert SYNC_FORMS.search(old)
    assert ASYNC_NULL.search("e = hipMemsetAsync(p, 0, 8, 0);")
    assert not ASYNC_NULL.search("e = hipMemsetAsync(p, 0, 8, c->s_in);")
    assert not SYNC_FORMS.search("hipMemsetAsync(c->arena, 0, n, c->s_in)")
