"""INTEGRATION.md's cgo binding, checked against include/*.h without a Go toolchain.

Go is absent from this image and from the GPU boxes, so the binding INTEGRATION.md
shows a maintainer is never built. This test does the part of `go build` that breaks
when the C ABI changes, with gcc:
- every `C.<name>` a Go block uses is declared by that file's cgo preamble (cgo
  resolves C names per file: a block without a preamble continues the first file);
- every call of a C function passes as many arguments as its prototype takes;
- every C struct field the Go code reads, sets or names in a composite literal exists;
- each preamble's own C (static helpers such as `replay_with_fields`) compiles.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")

# cgo's own pseudo-functions and its names for C's basic types
CGO_BUILTINS = {"GoString", "GoStringN", "GoBytes", "CString", "CBytes"}
CGO_BASIC = {"char", "schar", "uchar", "short", "ushort", "int", "uint", "long", "ulong", "longlong",
             "ulonglong", "float", "double", "size_t"}

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")


def go_blocks():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as fh:
        return re.findall(r"```go\n(.*?)```", fh.read(), re.S)


def split_preamble(block):
    """(preamble C text or None, cgo flags, Go code after the preamble)."""
    m = re.search(r"/\*\n(.*?)\*/\s*\nimport \"C\"\n", block, re.S)
    if not m:
        return None, [], block
    flags, lines = [], []
    for line in m.group(1).splitlines():
        d = re.match(r"\s*#cgo\s+(\w+):\s*(.*)", line)
        if d:
            if d.group(1) == "CFLAGS":
                flags += [f.replace("${SRCDIR}/../include", INC) for f in d.group(2).split()]
            continue
        lines.append(line)
    return "\n".join(lines) + "\n", flags, block[m.end():]


def files():
    """One entry per Go file: (name, preamble, cflags, Go code)."""
    out, first = [], None
    for k, block in enumerate(go_blocks()):
        pre, flags, code = split_preamble(block)
        if pre is None:
            if first is None:
                continue
            pre, flags = first
        elif first is None:
            first = (pre, flags)
        out.append(("go block %d" % (k + 1), pre, flags, code))
    return out


def compiles(pre, flags, body):
    with tempfile.NamedTemporaryFile("w", suffix=".c", delete=False) as fh:
        fh.write(pre + "\n#include <stddef.h>\n" + body + "\n")
        path = fh.name
    try:
        r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Werror", "-Wno-unused-function", "-I", INC] +
                           flags + [path], capture_output=True, text=True)
        return r.returncode == 0, r.stderr
    finally:
        os.unlink(path)


def strip_c_comments(s):
    return re.sub(r"/\*.*?\*/|//[^\n]*", " ", s, flags=re.S)


def balanced(s, i, open_ch, close_ch):
    """Index just past the bracket that closes s[i] (== open_ch)."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == open_ch:
            depth += 1
        elif s[j] == close_ch:
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced %s at %d" % (open_ch, i))


def top_level_split(s):
    parts, depth, cur, quote = [], 0, [], None
    for ch in s:
        if quote:
            cur.append(ch)
            if ch == quote:
                quote = None
            continue
        if ch in "\"'`":
            quote = ch
        elif ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
            continue
        cur.append(ch)
    if "".join(cur).strip():
        parts.append("".join(cur))
    return [p.strip() for p in parts]


def c_arity(decls, name):
    """Parameter count of C function `name` from its declaration/definition, or None."""
    for m in re.finditer(r"\b%s\s*\(" % re.escape(name), decls):
        open_at = m.end() - 1
        try:
            close = balanced(decls, open_at, "(", ")")
        except ValueError:
            continue
        tail = decls[close:close + 40].lstrip()
        before = decls[max(0, m.start() - 80):m.start()]
        # a declaration: a return type before the name, `;` or `{` after the list
        if (tail.startswith(";") or tail.startswith("{")) and re.search(r"[\w*]\s*$", before):
            params = decls[open_at + 1:close - 1].strip()
            return 0 if params in ("", "void") else len(top_level_split(params))
    return None


def header_text():
    out = []
    for f in sorted(os.listdir(INC)):
        if f.endswith(".h"):
            with open(os.path.join(INC, f)) as fh:
                out.append(fh.read())
    return strip_c_comments("\n".join(out))


def go_functions(code):
    """The Go code split at each top-level func (each function is its own scope)."""
    parts = re.split(r"\n(?=func )", "\n" + code)
    return [p for p in parts if p.strip()]


DECL = re.compile(r"\b([A-Za-z_]\w*(?:\s*,\s*[A-Za-z_]\w*)*)\s+(?:\*|\[\d*\])*C\.(\w+)")
ELEM = re.compile(r"\b(\w+)\s*:=\s*[\w.]*\.(\w+)\[[^\]]*\]")


def typed_names(code, elem_types):
    """Go identifiers declared with a C type in `code`: name -> C type name."""
    names = {}
    for m in DECL.finditer(code):
        for n in m.group(1).split(","):
            n = n.strip()
            if n not in ("var", "func", "return", "type"):
                names[n] = m.group(2)
    for m in ELEM.finditer(code):  # x := h.ci[k]: the element type of a slice field
        if m.group(2) in elem_types:
            names[m.group(1)] = elem_types[m.group(2)]
    for m in re.finditer(r"\b(\w+)\s*:=\s*C\.(\w+)\{", code):  # cr := C.gpk_results{...}
        names[m.group(1)] = m.group(2)
    return names


FILES = files()


@pytest.mark.parametrize("name,pre,flags,code", FILES, ids=[f[0].replace(" ", "_") for f in FILES])
def test_cgo_block_matches_headers(name, pre, flags, code):
    ok, err = compiles(pre, flags, "")
    assert ok, "%s: its cgo preamble does not compile:\n%s" % (name, err)
    problems = []

    # 1. every C.<name> resolves in this file's preamble (as a value or as a type)
    refs = sorted(set(re.findall(r"\bC\.(\w+)", code)) - CGO_BUILTINS - CGO_BASIC)
    kinds = {}
    for ref in refs:
        if compiles(pre, flags, "static void gpk_probe_(void) { (void)(%s); }" % ref)[0]:
            kinds[ref] = "value"
        elif compiles(pre, flags, "typedef %s gpk_probe_t;" % ref)[0]:
            kinds[ref] = "type"
        else:
            problems.append("C.%s is not declared by the preamble" % ref)

    # 2. calls pass as many arguments as the prototype takes
    decls = header_text() + strip_c_comments(pre)
    for m in re.finditer(r"\bC\.(\w+)\(", code):
        fn = m.group(1)
        if kinds.get(fn) != "value":
            continue
        want = c_arity(decls, fn)
        if want is None:  # libc / HIP runtime: declared, prototype not parsed here
            continue
        close = balanced(code, m.end() - 1, "(", ")")
        got = len(top_level_split(code[m.end():close - 1]))
        if got != want:
            problems.append("C.%s called with %d arguments, its prototype takes %d" % (fn, got, want))

    # 3. struct fields: composite literals and selectors on C-typed identifiers
    fields = set()
    for m in re.finditer(r"\bC\.(\w+)\{", code):
        close = balanced(code, m.end() - 1, "{", "}")
        for part in top_level_split(code[m.end():close - 1]):
            key = re.match(r"(\w+)\s*:", part)
            if key:
                fields.add((m.group(1), key.group(1)))
    elem_types = {}
    for m in DECL.finditer(code):  # Go struct fields of slice type: Records []C.gpk_record
        for n in m.group(1).split(","):
            elem_types[n.strip()] = m.group(2)
    for fn_code in go_functions(code):
        names = typed_names(fn_code, elem_types)
        for m in re.finditer(r"(?<![\w.])(\w+)\.([a-z_]\w*)", fn_code):
            var, field = m.groups()
            if var in names and var != "C":
                fields.add((names[var], field))
    for t, field in sorted(fields):
        if kinds.get(t) == "type" or compiles(pre, flags, "typedef %s gpk_probe_t;" % t)[0]:
            body = "static void gpk_probe_(void) { (void)sizeof(((%s*)0)->%s); }" % (t, field)
            if not compiles(pre, flags, body)[0]:
                problems.append("%s has no field %s" % (t, field))

    assert not problems, "%s:\n  %s" % (name, "\n  ".join(problems))


def test_every_go_block_is_checked():
    blocks = go_blocks()
    assert len(blocks) >= 6
    assert split_preamble(blocks[0])[0] is not None, "the first Go block must carry the package's preamble"
    assert len(files()) == len(blocks)
