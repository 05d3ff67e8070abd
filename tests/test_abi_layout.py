"""The ctypes mirror of the ABI structs (mpi-sppy_amd/_native.py) has the
layout of include/phx.h: a C probe compiled against the header prints the size
of every struct and the offset of every field the mirror names, and both must
agree (a field added on one side only shifts everything after it, silently)."""
import ctypes
import os
import re
import subprocess

import pytest

from mpisppy_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRUCTS = {
    "phx_problem_desc": _native.ProblemDesc,
    "phx_solve_opts": _native.SolveOpts,
    "phx_solve_stats": _native.SolveStats,
    "phx_tree_desc": _native.TreeDesc,
    "phx_iterk_args": _native.IterkArgs,
    "phx_iterk_result": _native.IterkResult,
}


def _probe(tmp_path):
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "phx.h"', "int main(void) {"]
    for cname, cls in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return dict((k, int(v)) for k, v in (ln.split() for ln in out.splitlines()))


def test_struct_layouts_match_header(tmp_path):
    c = _probe(tmp_path)
    for cname, cls in STRUCTS.items():
        for f in cls._fields_:
            assert getattr(cls, f[0]).offset == c["%s.%s" % (cname, f[0])], (cname, f[0])
        assert ctypes.sizeof(cls) == c[cname], cname


@pytest.mark.parametrize("cname", list(STRUCTS))
def test_no_header_field_missing(cname):
    """Every field the header declares in the struct is in the mirror."""
    text = open(os.path.join(ROOT, "include", "phx.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), text, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        m = re.search(r"\(\s*\*\s*(\w+)\s*\)", decl)       # function pointer
        if m:
            names.append(m.group(1))
            continue
        names += [re.sub(r"[\s*]", "", n) for n in decl.split(None, 1)[1].split(",")] if "," in decl \
            else [decl.replace("*", " ").split()[-1]]
    assert names == [f[0] for f in STRUCTS[cname]._fields_]
