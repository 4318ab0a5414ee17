"""INTEGRATION.md's code against include/pipck.h (CPU): every pipck_* call in
its C and Go blocks names a declared entry point with the header's number of
arguments, and the C blocks compile against the header (each bare identifier
declared with the type of the parameter it is passed as) -- so the binding a
maintainer copies from the document matches the ABI it describes."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "pipck.h"
DOC = ROOT / "INTEGRATION.md"


def _strip_comments(s: str) -> str:
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _split_top(args: str) -> list[str]:
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _prototypes() -> dict[str, list[str]]:
    """name -> parameter types (the declarator's name dropped)."""
    text = _strip_comments(HEADER.read_text())
    protos = {}
    for m in re.finditer(r"\b(pipck_\w+)\s*\(([^;{}]*?)\)\s*;", text, flags=re.S):
        params = _split_top(" ".join(m.group(2).split()))
        if params == ["void"]:
            params = []
        types = []
        for p in params:
            pm = re.match(r"(.*?[\s\*])(\w+)$", p)
            types.append((pm.group(1) if pm else p).strip())
        protos[m.group(1)] = types
    return protos


def _calls(block: str):
    """(name, [args]) for every pipck_* call in a code block."""
    text = _strip_comments(block)
    for m in re.finditer(r"\b(pipck_\w+)\s*\(", text):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        yield m.group(1), _split_top(text[m.end():i - 1])


def _blocks(lang: str) -> list[str]:
    return re.findall(r"```" + lang + r"\n(.*?)```", DOC.read_text(), flags=re.S)


def test_every_documented_call_matches_the_header():
    protos = _prototypes()
    assert "pipck_checksum_fixed_n" in protos and len(protos["pipck_checksum_fixed_n"]) == 11
    seen = 0
    for lang in ("c", "go"):
        for block in _blocks(lang):
            for name, args in _calls(block):
                assert name in protos, f"{name} is not declared in include/pipck.h"
                assert len(args) == len(protos[name]), (name, args, protos[name])
                seen += 1
    assert seen >= 8  # the TX, RX, update and cgo examples


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_c_examples_compile_against_the_header(tmp_path):
    protos = _prototypes()
    decls, bodies = {}, []
    for block in _blocks("c"):
        body = "\n".join(ln for ln in block.splitlines() if not ln.startswith("#include"))
        for name, args in _calls(body):
            for a, t in zip(args, protos[name]):
                if re.fullmatch(r"[A-Za-z_]\w*", a) and a != "NULL":
                    # drop top-level qualifiers: a variable usable for const and non-const parameters
                    decls.setdefault(a, re.sub(r"\bconst\b", "", t).strip())
        bodies.append(body)
    src = ['#include <stddef.h>', '#include "pipck.h"']
    src += [f"static {t} {v};" for v, t in sorted(decls.items())]
    for k, body in enumerate(bodies):
        src.append(f"int example_{k}(void) {{\n{body}\nreturn 0;\n}}")
    f = tmp_path / "integration_examples.c"
    f.write_text("\n".join(src) + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Wno-unused-value", "-Wno-unused-variable",
                        "-Werror=int-conversion", "-Werror=incompatible-pointer-types",
                        "-Werror=implicit-function-declaration", f"-I{ROOT / 'include'}", str(f)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr + "\n" + f.read_text()
