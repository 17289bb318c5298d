#!/usr/bin/env python3
"""Symbolise and attribute an nm03 CPU sample file (src/runtime/cpu_sampler.cpp, bench.py --cpu-profile).

    python tools/cpu_profile.py gpurun_out/prof/cpu.rank0 [--top 30] [--json out.json]

Frames are mapped to (module, ELF virtual address) through the recorded module map and the
modules' PT_LOAD headers, then named by llvm-symbolizer (inlined frames expanded: the build
carries host line tables). Reported:
  * samples per thread group (nm03-pool / nm03-slot / interpreter / runtime threads);
  * self time per function (innermost frame), per thread group;
  * the pool's time by task (a DICOM load, a JPEG-pair write, idle spinning, queue hand-off) and, for
    loads and writes, by phase: the first frame from the leaf that matches a phase's patterns.
"""
import argparse
import collections
import json
import os
import struct
import subprocess
import sys

SYMBOLIZER = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"

# (phase, substrings of a frame's function name), tried leaf-first per sample.
LOAD_PHASES = [
    ("open (path lookup)", ["__libc_open64", "open64", "__open64", "openat", "__GI___open"]),
    ("pread (page cache copy)", ["pread"]),
    ("close", ["__close", "close_nocancel", "__libc_close"]),
    ("12-bit pack", ["pack12::"]),
    ("DICOM parse", ["dicom::parse", "dicom::(anonymous namespace)", "Header"]),
    ("slot bookkeeping (locks, allocs, wakeups)", ["pthread_mutex", "lll_lock", "futex", "__lll", "notify_one",
                                                    "condition_variable", "load_into"]),
    ("string / alloc", ["malloc", "free", "operator new", "operator delete", "basic_string", "memcpy", "memmove"]),
]
WRITE_PHASES = [
    ("open/create", ["open64", "openat", "__libc_open64"]),
    ("pwritev/write", ["pwrite", "writev", "__libc_write", "__write"]),
    ("close", ["__close", "close_nocancel"]),
    ("ftruncate", ["ftruncate"]),
    ("path strings / alloc", ["malloc", "free", "operator new", "operator delete", "basic_string", "memcpy"]),
    ("other write work", ["write_jpeg_at", "jpeg::"]),
]


def load_phdrs(path, cache={}):
    """PT_LOAD (p_offset, p_vaddr, p_filesz) of an ELF64 file."""
    if path in cache:
        return cache[path]
    segs = []
    try:
        with open(path, "rb") as f:
            h = f.read(64)
            if h[:4] == b"\x7fELF" and h[4] == 2:
                phoff, = struct.unpack_from("<Q", h, 32)
                phentsize, phnum = struct.unpack_from("<HH", h, 54)
                f.seek(phoff)
                ph = f.read(phentsize * phnum)
                for i in range(phnum):
                    p_type, _flags, p_offset, p_vaddr, _paddr, p_filesz = struct.unpack_from("<IIQQQQ", ph, i * phentsize)
                    if p_type == 1:
                        segs.append((p_offset, p_vaddr, p_filesz))
    except OSError:
        pass
    cache[path] = segs
    return segs


def parse(path):
    """Returns meta, maps, threads, stacks [(count, tid, [pc...])] and rsi {stack index: rsi} (v2 files)."""
    maps, threads, stacks = [], {}, []
    meta = {"version": 1, "rsi": []}
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "#":
                if "v2" in line:
                    meta["version"] = 2
                continue
            if p[0] == "map":
                maps.append((int(p[1], 16), int(p[2], 16), int(p[3], 16), " ".join(p[4:])))
            elif p[0] == "thread":
                threads[int(p[1])] = p[2] if len(p) > 2 else "?"
            elif p[0] == "s":
                if meta["version"] >= 2:
                    meta["rsi"].append(int(p[3], 16))
                    stacks.append((int(p[1]), int(p[2]), [int(x, 16) for x in p[4:]]))
                else:
                    stacks.append((int(p[1]), int(p[2]), [int(x, 16) for x in p[3:]]))
            elif p[0] == "period_us":
                meta["period_us"] = int(p[1])
            elif p[0] == "samples":
                meta["samples"] = int(p[1])
                meta["dropped"] = int(p[3])
    return meta, maps, threads, stacks


def to_module(addr, maps):
    for lo, hi, off, path in maps:
        if lo <= addr < hi:
            foff = addr - lo + off
            for p_off, p_vaddr, p_sz in load_phdrs(path):
                if p_off <= foff < p_off + p_sz:
                    return path, p_vaddr + (foff - p_off)
            return path, foff
    return None, addr


def dynsym(path, cache={}):
    """Sorted (vaddr, name) of a module's dynamic symbols (stripped system libraries)."""
    if path not in cache:
        syms = []
        try:
            r = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, timeout=120)
            for line in r.stdout.splitlines():
                p = line.split()
                if len(p) == 3 and p[1] in "TtWi":
                    syms.append((int(p[0], 16), p[2].split("@")[0]))
        except (OSError, subprocess.TimeoutExpired, ValueError):
            pass
        cache[path] = sorted(syms)
    return cache[path]


def nearest_dynsym(path, a):
    syms = dynsym(path)
    lo, hi = 0, len(syms)
    while lo < hi:
        mid = (lo + hi) // 2
        if syms[mid][0] <= a:
            lo = mid + 1
        else:
            hi = mid
    if lo == 0:
        return None
    base, name = syms[lo - 1]
    # glibc 2.35: __lll_lock_wait / __lll_lock_wake (contended pthread mutexes, not exported) follow the
    # exported *_private variants; name them by their futex role.
    if name == "__lll_lock_wait_private" and a - base >= 0x60:
        return "__lll_lock_wait (futex wait, contended mutex)"
    if name == "__lll_lock_wake_private" and a - base >= 0x20:
        return "__lll_lock_wake (futex wake, contended mutex)"
    return f"{name}+{a - base:#x}"


def local_path(path, alias={}):
    """A module recorded on the GPU box (scratch checkout) → the same file in this checkout."""
    if os.path.exists(path):
        return path
    if path not in alias:
        here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        cand = os.path.join(here, "nm03_capstone_project_amd", "lib", os.path.basename(path))
        alias[path] = cand if "nm03_capstone_project_amd/lib/" in path and os.path.exists(cand) else path
    return alias[path]


def symbolize(requests):
    """{path: set(vaddr)} -> {(path, vaddr): [function names, innermost first]}."""
    out = {}
    for path, addrs in requests.items():
        obj = local_path(path)
        addrs = sorted(addrs)
        if not os.path.exists(obj):
            for a in addrs:
                out[(path, a)] = [f"{os.path.basename(path)}+{a:#x}"]
            continue
        inp = "".join(f"{a:#x}\n" for a in addrs)
        try:
            r = subprocess.run([SYMBOLIZER, f"--obj={obj}", "--functions=linkage", "--demangle", "--inlines",
                                "--output-style=JSON"], input=inp, capture_output=True, text=True, timeout=600)
            rows = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
        except (OSError, subprocess.TimeoutExpired, ValueError):
            rows = []
        for a, row in zip(addrs, rows):
            names = [s.get("FunctionName") or "??" for s in row.get("Symbol", [])]
            names = [n for n in names if n and n != "??"]
            if not names:
                nd = nearest_dynsym(obj, a)
                names = [nd] if nd else [f"{os.path.basename(path)}+{a:#x}"]
            out[(path, a)] = names
        for a in addrs:
            out.setdefault((path, a), [f"{os.path.basename(path)}+{a:#x}"])
    return out


# /usr/include/linux/kfd_ioctl.h: AMDKFD_IOC_* numbers ('K', nr); the size bits vary by struct.
KFD_IOCTL_NR = {0x01: "GET_VERSION", 0x02: "CREATE_QUEUE", 0x03: "DESTROY_QUEUE", 0x04: "SET_MEMORY_POLICY",
                0x05: "GET_CLOCK_COUNTERS", 0x06: "GET_PROCESS_APERTURES", 0x07: "UPDATE_QUEUE",
                0x08: "CREATE_EVENT", 0x09: "DESTROY_EVENT", 0x0A: "SET_EVENT", 0x0B: "RESET_EVENT",
                0x0C: "WAIT_EVENTS", 0x16: "ALLOC_MEMORY_OF_GPU", 0x17: "FREE_MEMORY_OF_GPU",
                0x18: "MAP_MEMORY_TO_GPU", 0x19: "UNMAP_MEMORY_FROM_GPU", 0x20: "GET_TILE_CONFIG"}


def kfd_ioctl_name(req):
    if (req >> 8) & 0xFF != ord("K"):
        return "not a KFD ioctl"
    return "AMDKFD_IOC_" + KFD_IOCTL_NR.get(req & 0xFF, f"nr {req & 0xFF:#x}")


def group_of(name):
    if name.startswith("nm03-pool"):
        return "nm03-pool"
    if name.startswith("nm03-slot"):
        return "nm03-slot"
    if name.startswith("nm03-reap"):
        return "nm03-reaper"
    if name.startswith("python"):
        return "main (python)"
    return "other: " + name


def classify(frames, phases):
    for fn in frames:
        for phase, pats in phases:
            if any(p in fn for p in pats):
                return phase
    return "other"


def analyse(path, top=30, chain_pat=""):
    meta, maps, threads, stacks = parse(path)
    req = collections.defaultdict(set)
    for _, _, pcs in stacks:
        for k, pc in enumerate(pcs):
            mod, va = to_module(pc if k == 0 else pc - 1, maps)  # return addresses: the call site
            if mod:
                req[mod].add(va)
    syms = symbolize(req)

    def frames_of(pcs):
        out = []
        for k, pc in enumerate(pcs):
            mod, va = to_module(pc if k == 0 else pc - 1, maps)
            out.extend(syms.get((mod, va), [f"{pc:#x}"]) if mod else [f"{pc:#x}"])
        return out

    total = sum(c for c, _, _ in stacks)
    lock_callers = collections.Counter()
    ioctls = collections.Counter()
    groups = collections.Counter()
    self_by_group = collections.defaultdict(collections.Counter)
    pool_task = collections.Counter()
    load_phase = collections.Counter()
    write_phase = collections.Counter()
    for si, (count, tid, pcs) in enumerate(stacks):
        g = group_of(threads.get(tid, "?"))
        groups[g] += count
        fr = frames_of(pcs)
        leaf = fr[0] if fr else "?"
        self_by_group[g][leaf] += count
        if leaf == "ioctl" and meta["rsi"]:
            ioctls[f"{g}: ioctl request {meta['rsi'][si]:#x} ({kfd_ioctl_name(meta['rsi'][si])})"] += count
        if any(f.startswith("__lll_lock") or f.startswith("__pthread_mutex") or "pthread_cond" in f for f in fr[:3]):
            # first frame of our code above the lock: who contends
            own = next((f for f in fr if "nm03::" in f or "ThreadPool" in f or "TaskGroup" in f or "Slot" in f
                        or "Engine" in f or "std::condition_variable" in f), fr[-1] if fr else "?")
            lock_callers[f"{g}: {leaf[:40]} <- {own[:110]}"] += count
        if g != "nm03-pool":
            continue
        joined = " | ".join(fr)
        if "load_into" in joined:
            pool_task["DICOM load"] += count
            load_phase[classify(fr, LOAD_PHASES)] += count
        elif "write_jpeg_at" in joined:
            pool_task["JPEG pair write"] += count
            write_phase[classify(fr, WRITE_PHASES)] += count
        elif "ThreadPool::loop" in joined and ("pause" in leaf or "steady_clock" in joined or "loop" in leaf):
            pool_task["idle spin (ThreadPool::loop)"] += count
        elif "TaskGroup" in joined or "ThreadPool" in joined:
            pool_task["queue hand-off (ThreadPool / TaskGroup)"] += count
        else:
            pool_task["other"] += count
    chains = collections.Counter()
    if chain_pat:
        for count, tid, pcs in stacks:
            fr = frames_of(pcs)
            if fr and any(chain_pat in f for f in fr[:2]):
                chains[" <- ".join(f[:60] for f in fr[:10])] += count
    res = {"file": path, "samples": total, "chains": chains.most_common(top), "period_us": meta.get("period_us"), "dropped": meta.get("dropped"),
           "groups": dict(groups.most_common()), "pool_task": dict(pool_task.most_common()),
           "load_phase": dict(load_phase.most_common()), "write_phase": dict(write_phase.most_common()),
           "self_top": {g: c.most_common(top) for g, c in self_by_group.items()},
           "lock_callers": lock_callers.most_common(top), "ioctls": ioctls.most_common(top)}
    return res


def report(res, out=sys.stdout):
    tot = max(res["samples"], 1)
    pct = lambda c, d=tot: f"{100.0 * c / max(d, 1):5.1f}%"
    print(f"{res['file']}: {res['samples']} samples (dropped {res['dropped']})", file=out)
    print("\nsamples by thread group:", file=out)
    for g, c in res["groups"].items():
        print(f"  {pct(c)}  {c:7d}  {g}", file=out)
    pool = res["groups"].get("nm03-pool", 0)
    if pool:
        print("\nnm03-pool by task (% of pool samples):", file=out)
        for t, c in res["pool_task"].items():
            print(f"  {pct(c, pool)}  {c:7d}  {t}", file=out)
        for title, key in (("DICOM load", "load_phase"), ("JPEG pair write", "write_phase")):
            sub = sum(res[key].values())
            if not sub:
                continue
            print(f"\n{title} by phase (% of its samples):", file=out)
            for t, c in res[key].items():
                print(f"  {pct(c, sub)}  {c:7d}  {t}", file=out)
    if res.get("chains"):
        print("\nfull call chains whose leaf frames match --chains (% of all samples):", file=out)
        for k, c in res["chains"]:
            print(f"  {pct(c)}  {c:7d}  {k}", file=out)
    if res.get("ioctls"):
        print("\nioctl samples by request code (% of all samples):", file=out)
        for k, c in res["ioctls"]:
            print(f"  {pct(c)}  {c:7d}  {k}", file=out)
    if res.get("lock_callers"):
        print("\nmutex / futex samples by caller (% of all samples):", file=out)
        for k, c in res["lock_callers"]:
            print(f"  {pct(c)}  {c:7d}  {k}", file=out)
    for g, rows in res["self_top"].items():
        gc = res["groups"].get(g, 1)
        print(f"\nself time, {g} (% of the group):", file=out)
        for fn, c in rows:
            print(f"  {pct(c, gc)}  {c:7d}  {fn[:150]}", file=out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json", default="")
    ap.add_argument("--chains", default="", help="also print the top full call chains whose leaf frames contain this")
    a = ap.parse_args()
    all_res = []
    for f in a.files:
        r = analyse(f, a.top, a.chains)
        report(r)
        all_res.append(r)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(all_res, f, indent=1)


if __name__ == "__main__":
    main()
