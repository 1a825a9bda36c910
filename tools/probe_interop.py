"""GPU-box probe: can libfmi_dev.so and torch share one HIP runtime in one process?

torch wheels bundle their own libamdhip64.so (soname libamdhip64.so.7) and librccl.so; libfmi_dev.so
is linked against /opt/rocm's copies. Importing torch first makes the dynamic linker bind
libfmi_dev.so to torch's already-loaded runtime (same soname). This probe checks which runtime files
get mapped and whether a kernel of ours runs correctly on a torch-allocated tensor and torch stream.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def mapped(substr):
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            if substr in line:
                out.add(line.split()[-1])
    return sorted(out)


def main():
    res = {}
    import torch  # noqa: F401  (first: its libamdhip64 wins the soname)

    res["torch"] = torch.__version__
    import fmi_amd

    fmi_amd.load()
    res["hip_runtimes_after_load"] = mapped("libamdhip64")
    res["rccl_after_load"] = mapped("librccl")
    res["torch_cuda"] = torch.cuda.is_available()
    fmi_amd.init(0)
    res["describe"] = fmi_amd.describe()
    n = (1 << 20) + 3
    a = torch.randn(n, device="cuda", dtype=torch.float32)
    b = torch.randn(n, device="cuda", dtype=torch.float32)
    want = a + b
    s = torch.cuda.current_stream().cuda_stream
    from fmi_amd import _lib
    _lib.call("fmi_dev_reduce_pair", 0, 0, a.data_ptr(), b.data_ptr(), n, s)
    torch.cuda.synchronize()
    res["torch_tensor_pair_ok"] = bool(torch.equal(a, want))
    res["hip_runtimes_after_use"] = mapped("libamdhip64")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
