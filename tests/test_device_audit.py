"""Static audit for the multi-GPU node: HIP's current device is per host thread and a new
thread starts on device 0, so on rank r of an 8-GPU node a PHY worker thread calling into the library would run on
GPU 0 unless every entry point selects its object's device itself.  Every exported function of the product libraries
(srsran_amd/csrc, srsran_amd/dropin) whose body does device work -- a HIP runtime call that allocates, copies,
launches, records or creates on the current device, a kernel-launch helper, a staging copy -- must first call
hipSetDevice, or first delegate to a function that does (another exported entry point, or a helper of the same file
that selects the device before its own device work).  The few entry points that act on the calling thread's device
by contract are listed with the reason."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = [os.path.join(ROOT, "srsran_amd", "csrc"), os.path.join(ROOT, "srsran_amd", "dropin")]

# calls that do not depend on (or change) the current device's state
NEUTRAL = ("SetDevice", "GetDevice", "GetDeviceCount", "GetLastError", "GetErrorString", "PointerGetAttributes",
           "EventQuery", "EventSynchronize", "EventElapsedTime", "EventDestroy", "HostFree", "StreamQuery",
           "StreamSynchronize", "StreamDestroy", "Free")
DEVICE_OP = re.compile(r"\bhip(?!(?:" + "|".join(NEUTRAL) + r")\s*\()[A-Z]\w*\s*\(|\b\w*launch\w*\s*\(|"
                       r"\bstage_copy\w*\s*\(|\bhipLaunchKernelGGL\b")
# entry points that use the calling thread's current device by contract
CURRENT_DEVICE = {
    "mi355_device_sync": "synchronises the calling thread's current device (its documented meaning)",
    "mi355_debug_stage_copy": "test hook: copies on the current device",
    "mi355_srslte_tdec_init_manual": "srslte_tdec_init_manual has no device argument: the decoder binds to the "
                                     "calling thread's current device, which it records for every later call",
}


def _strip(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _functions(src):
    """(name, body, exported) of every function definition starting at column 0"""
    out = []
    for m in re.finditer(r"^(static\s+|inline\s+)?[A-Za-z_][\w:<>\s\*&,]*?[\s\*&](\w+)\s*\(([^;{}]*)\)\s*(?:const\s*)?\{",
                         src, flags=re.M):
        i, depth = m.end(), 1
        while depth and i < len(src):
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        name = m.group(2)
        out.append((name, src[m.end():i], not m.group(1) and re.match(r"(mi355|srslte)_", name) is not None))
    return out


def _first(pattern, body):
    m = re.search(pattern, body)
    return m.start() if m else None


def _violations(fn, src):
    bad = []
    if True:
        if True:
            funcs = _functions(_strip(src))
            # helpers (any name) that select the device before any device work of their own
            setters = set()
            for name, body, _ in funcs:
                sd, op = _first(r"hipSetDevice\s*\(", body), _first(DEVICE_OP, body)
                if sd is not None and (op is None or sd < op):
                    setters.add(name)
            for name, body, exported in funcs:
                if not exported or name in CURRENT_DEVICE:
                    continue
                op = _first(DEVICE_OP, body)
                if op is None or name in setters:
                    continue
                calls = [m.start() for m in re.finditer(r"\b(\w+)\s*\(", body)
                         if m.group(1) in setters or re.match(r"(mi355|srslte)_", m.group(1))]
                if not calls or min(calls) > op:
                    bad.append(f"{fn}: {name} does device work before selecting its device: "
                               f"{body[op:op + 40].strip()!r}")
    return bad


def test_every_entry_point_selects_its_device():
    bad = []
    for d in DIRS:
        for fn in sorted(os.listdir(d)):
            if fn.endswith((".cpp", ".hip")):
                bad += _violations(fn, open(os.path.join(d, fn)).read())
    assert not bad, "\n".join(bad)


def test_audit_catches_a_missing_device_selection():
    src = """
static int helper(q_t* q) { CHECK_HIP(hipSetDevice(q->device)); return launch_x(q); }
int mi355_good(q_t* q) { int r = helper(q); hipMemcpyAsync(a, b, 4, hipMemcpyDeviceToHost, q->s); return r; }
int mi355_good2(q_t* q) { CHECK_HIP(hipSetDevice(q->device)); CHECK_HIP(hipMalloc(&q->p, 8)); return 0; }
int mi355_bad(q_t* q) { CHECK_HIP(hipMalloc(&q->p, 8)); CHECK_HIP(hipSetDevice(q->device)); return 0; }
int mi355_bad2(q_t* q) { if (!q) return 1; return tdec_launch_halfit(q->args, q->s); }
"""
    bad = _violations("sample.cpp", src)
    assert [b.split(":")[1].split()[0] for b in bad] == ["mi355_bad", "mi355_bad2"], bad
