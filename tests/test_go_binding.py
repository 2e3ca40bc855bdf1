"""The Go drop-in (go/graphing/nemohip.go) against the C ABI it binds
(include/nemohip.h): every C.nemo_* function it calls is declared with the same
number of parameters, every C.NEMO_* constant is #defined, every C.nemo_* type
is a typedef, and every field it touches on a C struct exists.  There is no Go
toolchain in this image, so this is the check that the file would link against
the header as written (reference call sites: main.go:33-44,95)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "graphing", "nemohip.go")
HDR = os.path.join(ROOT, "include", "nemohip.h")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", s, flags=re.S)


def _split_top(args):
    """Split an argument list at top-level commas."""
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def header_decls():
    h = _strip_c_comments(open(HDR).read())
    funcs = {}
    for m in re.finditer(r"\b([a-z_][a-z0-9_ ]*?[ *]+)(nemo_\w+)\s*\(([^;{]*?)\)\s*;", h):
        params = m.group(3).strip()
        funcs[m.group(2)] = 0 if params in ("", "void") else len(_split_top(params))
    defines = set(re.findall(r"^#define\s+(NEMO\w+)", h, flags=re.M))
    types = set(re.findall(r"typedef\s+struct\s+\w+\s*(?:\{.*?\})?\s*(nemo_\w+)\s*;", h, flags=re.S))
    fields = {}
    for m in re.finditer(r"typedef\s+struct\s+(nemo_\w+)\s*\{(.*?)\}\s*\w+\s*;", h, flags=re.S):
        fields[m.group(1)] = set(re.findall(r"(\w+)\s*(?:\[\d+\])?\s*;", m.group(2)))
    return funcs, defines, types, fields


def go_calls(src):
    """(name, argument count) of every C.nemo_*( call in the Go file."""
    calls = []
    for m in re.finditer(r"\bC\.(nemo_\w+)\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        args = src[m.end():i - 1]
        calls.append((m.group(1), len(_split_top(args)) if args.strip() else 0))
    return calls


def test_go_file_exists_and_is_the_graphing_package():
    src = open(GO).read()
    assert src.count("\npackage graphing\n") == 1
    assert '#include "nemohip.h"' in src and 'import "C"' in src
    # the ten GraphDatabase methods (main.go:33-44) on *Neo4J
    for name in ("InitGraphDB", "CloseDB", "LoadRawProvenance", "SimplifyProv", "CreatePrototypes",
                 "PullPrePostProv", "CreateNaiveDiffProv", "GenerateCorrections", "GenerateExtensions"):
        assert re.search(r"func \(n \*Neo4J\) %s\(" % name, src), name
    # CreateHazardAnalysis never touched Neo4j and stays in hazard-analysis.go (go/README.md)


def test_every_c_call_is_declared_with_matching_arity():
    funcs, _, types, _ = header_decls()
    src = open(GO).read()
    calls = go_calls(src)
    assert len(calls) > 20
    for name, n in calls:
        if name in types:  # a conversion such as C.nemo_chain(x) would count as a call
            continue
        assert name in funcs, f"{name} is not declared in include/nemohip.h"
        assert funcs[name] == n, f"{name}: Go passes {n} arguments, the header declares {funcs[name]}"


def test_every_c_constant_and_type_is_declared():
    _, defines, types, fields = header_decls()
    src = open(GO).read()
    for c in set(re.findall(r"\bC\.(NEMO_\w+)", src)):
        assert c in defines, f"C.{c} is not #defined in include/nemohip.h"
    for t in set(re.findall(r"\bC\.(nemo_\w+)\b(?!\()", src)):
        assert t in types, f"C.{t} is not a typedef in include/nemohip.h"
    # struct fields the binding reads or writes (`c` is a nemo_chain in SimplifyProv and a
    # *nemo_corpus in freeCorpus)
    for f in set(re.findall(r"\bcorpus\.(\w+)", src)):
        assert f in fields["nemo_corpus"], f"corpus.{f} is not a field of nemo_corpus"
    for f in set(re.findall(r"\bc\.(\w+)", src)):
        assert f in fields["nemo_corpus"] | fields["nemo_chain"], f"c.{f} is not a field of nemo_corpus/nemo_chain"
    for f in set(re.findall(r"\brow\.(\w+)", src)):
        assert f in fields["nemo_missing"], f"row.{f} is not a field of nemo_missing"


def test_header_parser_sees_the_whole_abi():
    funcs, defines, types, _ = header_decls()
    assert funcs["nemo_fetch_triggers"] == 10 and funcs["nemo_abi_version"] == 0
    assert funcs["nemo_protos_finalize"] == 9 and funcs["nemo_ctx_create_node"] == 3
    assert {"nemo_ctx", "nemo_corpus", "nemo_chain", "nemo_missing"} <= types
    assert {"NEMO_OK", "NEMO_DIFF_REFERENCE", "NEMO_F_HOLDS"} <= defines
