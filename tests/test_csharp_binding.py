"""The C# P/Invoke binding (bindings/csharp/TrueTraceHip.cs) is shipped but cannot be compiled
here (no .NET runtime in the image or on the GPU box). What can be checked without it: every
[DllImport] entry point is exported by the built library, and the binding's flag values equal the
header's."""
import os
import re

import tthip

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = open(os.path.join(REPO, "bindings", "csharp", "TrueTraceHip.cs")).read()
HDR = open(os.path.join(REPO, "include", "truetrace_hip.h")).read()


def test_every_dllimport_is_exported():
    L = tthip.hip_lib()
    names = set()
    for m in re.finditer(r'\[DllImport\(Lib(?:,\s*EntryPoint\s*=\s*"(\w+)")?\)\][^;]*?\bextern\b[^(]*?\b(\w+)\s*\(', CS, re.S):
        names.add(m.group(1) or m.group(2))
    assert len(names) >= 18, names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def _header_functions():
    src = re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(tt_[a-z0-9_]+)\s*\(", src, flags=re.M)))


def _bound():
    names = set()
    for m in re.finditer(r'\[DllImport\(Lib(?:,\s*EntryPoint\s*=\s*"(\w+)")?\)\][^;]*?\bextern\b[^(]*?\b(\w+)\s*\(', CS, re.S):
        names.add(m.group(1) or m.group(2))
    return names


# header functions a C# host has no use for, with the reason (everything else must have a [DllImport])
HOST_ONLY = {}


def test_every_header_function_is_bound_or_listed_host_only():
    hdr = _header_functions()
    assert "tt_group_trace_frame" in hdr and "tt_shutdown" in hdr
    unbound = [n for n in hdr if n not in _bound() and n not in HOST_ONLY]
    assert not unbound, unbound
    assert not (set(HOST_ONLY) - set(hdr)), "stale HOST_ONLY entries"


def test_group_flags_match_header():
    cs = dict(re.findall(r"(CopyGather|Bounce|Info)\s*=\s*1u\s*<<\s*(\d+)", CS))
    hdr = dict(re.findall(r"(TT_GROUP_\w+)\s*=\s*1u\s*<<\s*(\d+)", HDR))
    assert cs["CopyGather"] == hdr["TT_GROUP_COPY_GATHER"] and cs["Bounce"] == hdr["TT_GROUP_BOUNCE"]
    assert cs["Info"] == hdr["TT_GROUP_INFO"]


def test_flag_values_match_header():
    cs = {k: int(v) for k, v in re.findall(r"(\w+)\s*=\s*1u\s*<<\s*(\d+)", CS)}
    hdr = {k: int(v) for k, v in re.findall(r"(TT_(?:TRACE|SHADOW)_\w+)\s*=\s*1u\s*<<\s*(\d+)", HDR)}
    pairs = {"DevicePtrs": "TT_TRACE_DEVICE_PTRS", "UseReSTIRGI": "TT_TRACE_USE_RESTIRGI",
             "UseASVGF": "TT_TRACE_USE_ASVGF", "Stats": "TT_TRACE_STATS", "Async": "TT_TRACE_ASYNC",
             "IgnoreGlass": "TT_TRACE_IGNORE_GLASS", "IgnoreBackfacing": "TT_TRACE_IGNORE_BACKFACING",
             "AdaptiveOrder": "TT_TRACE_ADAPTIVE_ORDER",
             "RadianceCache": "TT_SHADOW_RADIANCE_CACHE", "VisibilityCheck": "TT_SHADOW_VISIBILITY_CHECK"}
    for c, h in pairs.items():
        assert cs[c] == hdr[h], (c, h)
