"""Static checks of the cgo binding (pkg/fitgpu) against the C-ABI header: this image has no Go
toolchain, so these guard the binding's text.  Every `C.fit_*` function the Go code calls is
declared in include/fitgpu.h, and every field of `fit_admit_req` crosses the binding both ways
(cReq sets it, PodDemand copies it back) — a field the Go side drops is silently zero on the C side
(round 5: the array flag, without which the Go call site pinned array tasks to one node)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "fitgpu.h")
GO = os.path.join(ROOT, "slurm-bridge-operator_amd", "pkg", "fitgpu")


def _go_sources():
    out = {}
    for f in sorted(os.listdir(GO)):
        if f.endswith(".go"):
            with open(os.path.join(GO, f)) as fh:
                out[f] = fh.read()
    return out


def _header():
    with open(HDR) as fh:
        return fh.read()


def _struct_fields(hdr, name):
    end = re.search(r"\}\s*" + name + r"\s*;", hdr)
    assert end, name
    start = hdr.rfind("typedef struct", 0, end.start())
    body = hdr[hdr.index("{", start) + 1:end.start()]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:
            fields.append(re.split(r"[\s*]+", decl)[-1].split("[")[0])
    return fields


def test_every_called_function_is_declared():
    hdr = _header()
    declared = set(re.findall(r"\b(fit_[a-z0-9_]+)\s*\(", hdr))
    called = set()
    for text in _go_sources().values():
        called |= set(re.findall(r"\bC\.(fit_[a-z0-9_]+)\s*\(", text))
    assert called, "no cgo calls found"
    assert called <= declared, sorted(called - declared)


def test_admit_request_fields_cross_both_ways():
    hdr = _header()
    fields = [f for f in _struct_fields(hdr, "fit_admit_req") if f != "reserved"]
    src = "\n".join(_go_sources().values())
    creq = re.search(r"func cReq\(d Demand\) C\.fit_admit_req \{(.*?)\n\}", src, re.S)
    assert creq, "cReq not found"
    for f in fields:
        assert re.search(r"\b" + f + r"\s*:", creq.group(1)), f"cReq does not set {f}"
    back = re.search(r"out\[i\] = Demand\{(.*?)\}", src, re.S)
    assert back, "PodDemand's copy not found"
    for f in fields:
        assert re.search(r"\br\." + f + r"\b", back.group(1)), f"PodDemand does not copy {f}"
