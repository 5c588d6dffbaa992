"""Which HIP / HSA runtime does a process map when it uses both the engine
(libemqx_tm.so, linked against /opt/rocm) and torch (bundled ROCm runtime)?

    python tools/probe_runtime.py engine_first|torch_first|host

Prints the mapped libamdhip64 / libhsa-runtime64 files and whether each side
sees the GPU.  `host` prints the CPU share of this lease (affinity, cgroup
quota, model, clocks).  Dev tool: evidence for DESIGN.md §8.
"""

import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def maps():
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if "libamdhip64" in p or "libhsa-runtime64" in p or "librccl" in p:
                out.add(p)
    return sorted(out)


def engine_devices():
    from emqx_amd import _native as N
    return N.lib().tm_device_count()


def host():
    print("os.cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpuset.cpus.effective"):
        try:
            with open(p) as f:
                print(p, f.read().strip())
        except OSError as e:
            print(p, "n/a", e.__class__.__name__)
    with open("/proc/cpuinfo") as f:
        seen = set()
        for line in f:
            k = line.split(":")[0].strip()
            if k in ("model name", "cpu MHz") and k not in seen:
                print(line.strip())
                seen.add(k)
    for p in ("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq",
              "/sys/devices/system/cpu/cpu0/cpufreq/scaling_cur_freq"):
        try:
            with open(p) as f:
                print(p, f.read().strip())
        except OSError:
            print(p, "n/a")


def main():
    mode = sys.argv[1]
    if mode == "host":
        return host()
    if mode == "engine_first":
        print("engine devices:", engine_devices())
        print("maps after engine:", maps())
        import torch
        print("maps after import torch:", maps())
        try:
            print("torch.cuda.device_count:", torch.cuda.device_count())
            torch.cuda.init()
            x = torch.ones(4, device="cuda:0")
            print("torch tensor ok:", float(x.sum()))
        except Exception as e:  # the round-1 symptom
            print("torch cuda init failed:", repr(e))
        print("maps at end:", maps())
    else:
        import torch
        x = torch.ones(4, device="cuda:0")
        print("torch tensor ok:", float(x.sum()))
        print("maps after torch init:", maps())
        print("engine devices:", engine_devices())
        from emqx_amd.engine import Engine
        e = Engine(device=0)
        e.insert(b"a/+/c")
        offs, ids = e.match_batch([b"a/b/c", b"x"])
        print("engine match after torch:", list(offs), list(ids))
        print("maps at end:", maps())
        y = torch.ones(4, device="cuda:0") * 2
        print("torch still ok:", float(y.sum()))


if __name__ == "__main__":
    main()
