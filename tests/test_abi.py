"""CPU-side checks of the drop-in boundary: the library loads and exports every
symbol include/ksg.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "ksg.h")


def declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(ksg_\w+)\(", txt, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("ksg_create", "ksg_load_cluster", "ksg_schedule_queue", "ksg_pod_results",
                 "ksg_annotations", "ksg_filter_codes", "ksg_scores", "ksg_cycle", "ksg_reserve",
                 "ksg_unreserve"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from ksg import load_library
    L = load_library()
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version():
    from ksg import load_library
    L = load_library()
    assert L.ksg_abi_version() == 4
