"""Which HIP stream does torch's "stream 0" launch on? A spin kernel (~1 s) goes on
torch.cuda.ExternalStream(0) and on torch's default current stream; while it runs,
hipStreamQuery is asked (through the same libamdhip64 torch loaded) about the legacy null
stream (handle 0) and the per-thread default stream (handle 2). hipErrorNotReady (600) means
that stream has the spin queued. This decides whether torch's work can hold back a
null-stream hipMemset issued by a library in the same process (round-6 memset race,
profiles/r06/intermittent/README.md §6)."""
import ctypes
import json
import time

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")  # already loaded by torch: the same runtime
    hip.hipStreamQuery.restype = ctypes.c_int
    hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
    torch.cuda.init()
    torch.cuda.synchronize()
    out = {"torch_current_stream": int(torch.cuda.current_stream().cuda_stream)}
    for label, stream in (("ExternalStream(0)", torch.cuda.ExternalStream(0)), ("current", None)):
        torch.cuda.synchronize()
        if stream is None:
            torch.cuda._sleep(2_000_000_000)
        else:
            with torch.cuda.stream(stream):
                torch.cuda._sleep(2_000_000_000)
        time.sleep(0.01)
        out[label] = {"query_null(0)": hip.hipStreamQuery(None), "query_per_thread(2)": hip.hipStreamQuery(ctypes.c_void_p(2)),
                      "torch_query": torch.cuda.current_stream().query() if stream is None else stream.query()}
        torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
