"""Static check of the driver-facing scripts on CPU: every global name bench.py and
__graft_entry__.py read is defined or imported (a NameError there would only show on the GPU box)."""
import builtins
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _undefined_globals(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    defined = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    defined |= set(dir(builtins)) | {"__file__", "__name__"}
    bad = set()

    def walk(t):
        for s in t.get_symbols():
            if s.is_global() and s.is_referenced() and s.get_name() not in defined:
                bad.add((t.get_name(), s.get_name()))
        for c in t.get_children():
            walk(c)
    walk(top)
    return bad


@pytest.mark.parametrize("script", ["bench.py", "__graft_entry__.py", "profiles/scripts/c5_only.py",
                                    "profiles/scripts/match_only.py", "profiles/scripts/extract_only.py"])
def test_no_undefined_globals(script):
    assert not _undefined_globals(os.path.join(ROOT, script))
