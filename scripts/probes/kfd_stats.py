"""KFD's per-process counters (sysfs), for the walk probes."""
import os


def kfd_self():
    """KFD's counters of every process holding a GPU (the container's pid
    namespace hides which host pid is ours: the caller takes the one whose
    VRAM holds this process's planes): pid -> evicted_ms, vram GiB, page moves."""
    base = "/sys/class/kfd/kfd/proc"
    out = {}
    try:
        pids = os.listdir(base)
    except OSError:
        return None
    for pid in pids:
        d = os.path.join(base, pid)
        r = {"evicted_ms": 0, "vram_gib": 0.0, "page_in": 0, "page_out": 0}
        try:
            for e in os.listdir(d):
                if e.startswith("stats_"):
                    r["evicted_ms"] += int(open(os.path.join(d, e, "evicted_ms")).read())
                elif e.startswith("vram_"):
                    r["vram_gib"] += int(open(os.path.join(d, e)).read()) / 2**30
                elif e.startswith("counters_"):
                    r["page_in"] += int(open(os.path.join(d, e, "page_in")).read())
                    r["page_out"] += int(open(os.path.join(d, e, "page_out")).read())
        except (OSError, ValueError):
            continue
        out[pid] = r
    return out
