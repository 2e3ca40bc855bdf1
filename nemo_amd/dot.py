"""DOT graphs with the observable behaviour of the gographviz revision the reference
vendors (vendor/github.com/awalterschulze/gographviz, rev c45f112): the type
the `graphing` package returns to main.go and the report.

Graph model (graph.go, nodes.go, edges.go, relations.go, subgraphs.go):
* ``add_node`` of an existing name extends its attributes, overwriting equal
  keys (nodes.go:39-47); ``nodes`` keeps first-insertion order (the
  ``Nodes.Nodes`` slice createDiffDot iterates).
* Edges keep insertion order; ``src_to_dsts`` indexes them like
  ``Edges.SrcToDsts`` (edges.go).
* Every node / subgraph records its parent graph (``Relations``).

Writer (write.go:118-154, ast/ast.go): ``[strict ]digraph|graph NAME {``, then
the graph attributes (sorted), every edge in insertion order, the main graph's
unwritten subgraphs (sorted) and finally every node not yet written inside a
subgraph (sorted), each as a tab-indented statement ending in ``;``, then
``\\n}\\n``.  Attribute lists are sorted and written ``[ k=v, k=v ]``; IDs are
verbatim (quoted strings keep their quotes).  Ports are dropped on output (the
reference passes ``Port.String()``, which starts with ':', back into
``MakeNodeID``, whose first ':'-field is then empty — write.go:66-69).

Reader (``read_dot``, gographviz.Read = parser + analyse.go): the full DOT
grammar of the vendored parser (internal/parser/productionstable.go), with
node/edge default attribute statements applied the way analyse.go applies them.
Anonymous subgraphs are named ``anon<N>`` with a counter (the reference draws a
random number, ast.go:186).  The reference also rejects attribute names outside
Graphviz's list (attr.go); this reader accepts any name.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Tuple


class Edge:
    __slots__ = ("src", "dst", "directed", "attrs")

    def __init__(self, src: str, dst: str, directed: bool, attrs: Dict[str, str]):
        self.src, self.dst, self.directed, self.attrs = src, dst, directed, dict(attrs)


class DotGraph:
    def __init__(self, name: str = "", directed: bool = True, strict: bool = False):
        self.name = name
        self.directed = directed
        self.strict = strict
        self.attrs: Dict[str, str] = {}
        self.nodes: Dict[str, Dict[str, str]] = {}  # name -> attrs, first-insertion order
        self.edges: List[Edge] = []
        self.src_to_dsts: Dict[Tuple[str, str], List[Edge]] = {}
        self.subgraphs: Dict[str, Dict[str, str]] = {}  # name -> attrs
        self.children: Dict[str, set] = {}              # Relations.ParentToChildren

    # graph.go:69-98
    def add_node(self, parent: str, name: str, attrs: Dict[str, str]) -> None:
        if name in self.nodes:
            self.nodes[name].update(attrs)
        else:
            self.nodes[name] = dict(attrs)
        self.children.setdefault(parent, set()).add(name)

    def add_edge(self, src: str, dst: str, directed: bool, attrs: Dict[str, str]) -> None:
        e = Edge(src, dst, directed, attrs)
        self.edges.append(e)
        self.src_to_dsts.setdefault((src, dst), []).append(e)

    def add_attr(self, parent: str, field: str, value: str) -> None:
        if parent == self.name:
            self.attrs[field] = value
        elif parent in self.subgraphs:
            self.subgraphs[parent][field] = value
        else:
            raise KeyError(f"graph or subgraph {parent} does not exist")

    def add_subgraph(self, parent: str, name: str, attrs: Dict[str, str]) -> None:
        self.children.setdefault(parent, set()).add(name)
        self.subgraphs.setdefault(name, {})
        for k, v in attrs.items():
            self.add_attr(name, k, v)

    # ---- writer ----------------------------------------------------------------
    @staticmethod
    def _attr_list(attrs: Dict[str, str]) -> str:
        if not attrs:
            return ""
        return "[ " + ", ".join(f"{k}={attrs[k]}" for k in sorted(attrs)) + " ] "

    @staticmethod
    def _stmts(stmts: List[str]) -> str:
        return "".join("\t" + s + ";\n" for s in stmts if s)

    def _node_stmt(self, name: str, written: set) -> str:
        written.add(name)
        return (name + " " + self._attr_list(self.nodes[name])).strip()

    def _subgraph_stmt(self, name: str, written: set) -> str:
        written.add(name)
        stmts = [f"{k}={v}" for k, v in sorted(self.subgraphs[name].items())]
        for child in sorted(self.children.get(name, ())):
            if child in self.nodes:
                stmts.append(self._node_stmt(child, written))
            elif child in self.subgraphs:
                stmts.append(self._subgraph_stmt(child, written))
            else:
                raise KeyError(f"{child} is not a node or a subgraph")
        return "subgraph " + name + " {\n" + self._stmts(stmts) + "\n}\n"

    def _location(self, name: str, written: set) -> str:
        if name in self.nodes:
            return name
        if name in self.subgraphs:
            return name if name.startswith("cluster") else self._subgraph_stmt(name, written)
        raise KeyError(f"{name} is not a node or a subgraph")

    def string(self) -> str:
        written: set = set()
        stmts: List[str] = [f"{k}={self.attrs[k]}" for k in sorted(self.attrs)]
        for e in self.edges:
            src = self._location(e.src, written)
            dst = self._location(e.dst, written)
            op = "->" if e.directed else "--"
            stmts.append((src + (op + dst).strip() + self._attr_list(e.attrs)).strip())
        top = self.children.get(self.name, set())
        for s in sorted(self.subgraphs):
            if s not in written and s in top:
                stmts.append(self._subgraph_stmt(s, written))
        for name in sorted(self.nodes):
            if name not in written:
                stmts.append(self._node_stmt(name, written))
        head = ("strict " if self.strict else "") + ("digraph " if self.directed else "graph ")
        return head + self.name + " {\n" + self._stmts(stmts) + "\n}\n"

    __str__ = string


# ---- reader ------------------------------------------------------------------------
class DotSyntaxError(ValueError):
    pass


_KEYWORDS = {"graph", "digraph", "node", "edge", "strict", "subgraph"}
_TOKEN = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/|^\#[^\n]*) |
    (?P<op>->|--|[{}\[\];=,:]) |
    (?P<str>"(?:[^"\\]|\\.)*") |
    (?P<num>-?(?:\.[0-9]+|[0-9]+(?:\.[0-9]*)?)) |
    (?P<id>[A-Za-z_\x80-\U0010FFFF][A-Za-z_0-9\x80-\U0010FFFF]*) |
    (?P<html><)
""", re.X | re.S | re.M)


def _tokens(text: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    i, n = 0, len(text)
    while i < n:
        m = _TOKEN.match(text, i)
        if not m:
            raise DotSyntaxError(f"unexpected character {text[i]!r} at offset {i}")
        kind = m.lastgroup
        if kind == "html":
            depth, j = 0, i
            while j < n:
                if text[j] == "<":
                    depth += 1
                elif text[j] == ">":
                    depth -= 1
                    if depth == 0:
                        break
                j += 1
            if j >= n:
                raise DotSyntaxError("unterminated HTML string")
            out.append(("id", text[i:j + 1]))
            i = j + 1
            continue
        if kind == "id" and m.group(kind).lower() in _KEYWORDS and m.group(kind) in (
                m.group(kind).lower(), m.group(kind).capitalize(), m.group(kind).upper()):
            out.append(("kw", m.group(kind).lower()))
        elif kind in ("str", "num", "id"):
            out.append(("id", m.group(kind)))
        elif kind == "op":
            out.append(("op", m.group(kind)))
        i = m.end()
    return out


class _Parser:
    """Recursive-descent parser for the grammar of productionstable.go, driving the
    analyse.go visitor semantics as it goes."""

    def __init__(self, text: str):
        self.t = _tokens(text)
        self.i = 0
        self.anon = 0
        self.g: Optional[DotGraph] = None

    def peek(self, k: int = 0) -> Tuple[str, str]:
        return self.t[self.i + k] if self.i + k < len(self.t) else ("eof", "")

    def take(self, kind: str, val: Optional[str] = None) -> str:
        tk = self.peek()
        if tk[0] != kind or (val is not None and tk[1] != val):
            raise DotSyntaxError(f"expected {val or kind}, got {tk[1] or tk[0]!r}")
        self.i += 1
        return tk[1]

    def at(self, kind: str, val: Optional[str] = None) -> bool:
        tk = self.peek()
        return tk[0] == kind and (val is None or tk[1] == val)

    def graph(self) -> DotGraph:
        strict = False
        if self.at("kw", "strict"):
            self.i += 1
            strict = True
        if self.at("kw", "digraph"):
            directed = True
        elif self.at("kw", "graph"):
            directed = False
        else:
            raise DotSyntaxError("expected graph or digraph")
        self.i += 1
        name = self.take("id") if self.at("id") else ""
        self.g = DotGraph(name, directed, strict)
        self.take("op", "{")
        self.stmt_list(name, {}, {})
        self.take("op", "}")
        if not self.at("eof"):
            raise DotSyntaxError("trailing input after graph")
        return self.g

    # analyse.go:56-62: a statement scope carries node/edge defaults and created nodes
    def stmt_list(self, gname: str, node_defaults: Dict[str, str], edge_defaults: Dict[str, str]) -> None:
        scope = {"g": gname, "node": dict(node_defaults), "edge": dict(edge_defaults), "graph": {}, "created": set()}
        while not self.at("op", "}"):
            if self.at("eof"):
                raise DotSyntaxError("unexpected end of input")
            self.stmt(scope)
            if self.at("op", ";"):
                self.i += 1

    def attr_list(self) -> Dict[str, str]:
        attrs: Dict[str, str] = {}
        while self.at("op", "["):
            self.i += 1
            while not self.at("op", "]"):
                k = self.take("id")
                v = "true"
                if self.at("op", "="):
                    self.i += 1
                    v = self.take("id")
                attrs[k] = v
                if self.at("op", ",") or self.at("op", ";"):
                    self.i += 1
            self.take("op", "]")
        return attrs

    def stmt(self, sc: dict) -> None:
        g = self.g
        if self.at("kw", "graph") or self.at("kw", "node") or self.at("kw", "edge"):
            kw = self.take("kw")
            attrs = self.attr_list()
            if kw == "node":
                sc["node"].update(attrs)
            elif kw == "edge":
                sc["edge"].update(attrs)
            else:
                for k, v in attrs.items():
                    g.add_attr(sc["g"], k, v)
                sc["graph"].update(attrs)
            return
        if self.at("id") and self.peek(1) == ("op", "="):
            k = self.take("id")
            self.i += 1
            g.add_attr(sc["g"], k, self.take("id"))
            return
        src, src_is_node = self.location(sc)
        if self.at("op", "->") or self.at("op", "--"):
            rhs = []
            while self.at("op", "->") or self.at("op", "--"):
                directed = self.take("op") == "->"
                rhs.append((directed,) + self.location(sc))
            attrs = self.attr_list()
            for k, v in sc["edge"].items():
                attrs.setdefault(k, v)
            if src_is_node:
                self._node_from_edge(sc, src)
            for directed, dst, dst_is_node in rhs:
                if dst_is_node:
                    self._node_from_edge(sc, dst)
                g.add_edge(src, dst, directed, attrs)
                src = dst
            return
        if not src_is_node:
            return  # a bare subgraph statement
        attrs = self.attr_list()
        if src not in sc["created"]:
            sc["created"].add(src)
            for k, v in sc["node"].items():
                attrs.setdefault(k, v)
        g.add_node(sc["g"], src, attrs)

    def _node_from_edge(self, sc: dict, name: str) -> None:
        if name not in sc["created"]:
            sc["created"].add(name)
            self.g.add_node(sc["g"], name, sc["node"])

    def location(self, sc: dict) -> Tuple[str, bool]:
        if self.at("kw", "subgraph") or self.at("op", "{"):
            name = ""
            if self.at("kw", "subgraph"):
                self.i += 1
                if self.at("id"):
                    name = self.take("id")
            if not name:
                name = f"anon{self.anon}"
                self.anon += 1
            self.g.add_subgraph(sc["g"], name, sc["graph"])
            self.take("op", "{")
            self.stmt_list(name, sc["node"], sc["edge"])
            self.take("op", "}")
            return name, False
        name = self.take("id")
        if self.at("op", ":"):  # port: parsed, then lost on output (module docstring)
            self.i += 1
            self.take("id")
            if self.at("op", ":"):
                self.i += 1
                self.take("id")
        return name, True


def read_dot(text: str) -> DotGraph:
    """gographviz.Read (gographviz.go:52-58)."""
    return _Parser(text).graph()


# ---- createDOT / createDiffDot ------------------------------------------------------
class ProvNode:
    """The node properties createDOT reads from a DUETO path end
    (graph.Node.Properties / Labels of the Bolt driver)."""
    __slots__ = ("id", "label", "table", "type", "holds", "is_rule", "time")

    def __init__(self, id: str, label: str, table: str, type: Optional[str], holds: Optional[bool], is_rule: bool,
                 time: str = ""):
        self.id, self.label, self.table, self.type = id, label, table, type
        self.holds, self.is_rule, self.time = holds, is_rule, time

    def __repr__(self) -> str:
        return f"ProvNode({self.id!r})"


def _node_attrs(n: ProvNode, graph_type: str) -> Dict[str, str]:
    a = {"label": f'"{n.label}"', "style": '"filled, solid"', "color": '"black"', "fontcolor": '"black"',
         "fillcolor": '"white"'}
    if n.type == "async":
        a["style"] = '"filled, bold"'
        a["color"] = '"lawngreen"'
    elif n.type == "next":
        a["fontcolor"] = '"gold"'
    if n.holds is True and graph_type == "pre":
        a["color"] = '"firebrick"'
        a["fillcolor"] = '"firebrick"'
    elif n.holds is True and graph_type == "post":
        a["color"] = '"deepskyblue"'
        a["fillcolor"] = '"deepskyblue"'
    a["shape"] = "rect" if n.is_rule else "ellipse"
    return a


def create_dot(edges: List[Tuple[ProvNode, ProvNode]], graph_type: str) -> DotGraph:
    """createDOT (graphing/diagrams.go:15-130)."""
    g = DotGraph("dataflow", True)
    g.add_node("dataflow", "graph", {"bgcolor": '"transparent"'})
    for f, t in edges:
        g.add_node("dataflow", f.id, _node_attrs(f, graph_type))
        g.add_node("dataflow", t.id, _node_attrs(t, graph_type))
        g.add_edge(f.id, t.id, True, {"color": '"black"'})
    return g


def create_diff_dot(diff_run: int, diff_edges: List[Tuple[ProvNode, ProvNode]],
                    failed_edges: List[Tuple[ProvNode, ProvNode]], success_run: int, success_post: DotGraph,
                    missing_ids: set) -> Tuple[DotGraph, DotGraph]:
    """createDiffDot (graphing/diagrams.go:133-291); `missing_ids` = every Missing
    rule ID and goal ID (the missingMap of :136-144)."""
    diff = DotGraph("dataflow", True)
    failed = DotGraph("dataflow", True)
    for g in (diff, failed):
        g.add_node("dataflow", "graph", {"bgcolor": '"transparent"'})
    old, new = f"run_{success_run}", f"run_{diff_run}"
    for e in success_post.edges:
        a = dict(e.attrs)
        a["style"] = '"invis"'
        for g in (diff, failed):
            g.add_edge(e.src.replace(old, new), e.dst.replace(old, new), e.directed, a)
    for name, attrs in success_post.nodes.items():
        a = dict(attrs)
        a["style"] = '"invis"'
        for g in (diff, failed):
            g.add_node("dataflow", name.replace(old, new), a)
    for f, t in diff_edges:
        diff.nodes[f.id]["style"] = '"filled, solid"'
        diff.nodes[t.id]["style"] = '"filled, solid"'
        for e in diff.src_to_dsts.get((f.id, t.id), []):
            e.attrs["style"] = '"filled, solid"'
        if f.id in missing_ids:
            diff.nodes[f.id]["style"] = '"filled, dashed, bold"'
            diff.nodes[f.id]["color"] = '"mediumvioletred"'
        if t.id in missing_ids:
            diff.nodes[t.id]["style"] = '"filled, dashed, bold"'
            diff.nodes[t.id]["color"] = '"mediumvioletred"'
    labels = set()
    for f, t in failed_edges:
        labels.add(f'"{f.label}"')
        labels.add(f'"{t.label}"')
    for attrs in failed.nodes.values():  # :267-277 (one pass over the label set instead of E_fail passes)
        if attrs.get("label") in labels:
            attrs["style"] = '"filled, solid"'
    solid = '"filled, solid"'
    for e in failed.edges:
        if failed.nodes[e.src].get("style") == solid and failed.nodes[e.dst].get("style") == solid:
            e.attrs["style"] = solid
    return diff, failed
