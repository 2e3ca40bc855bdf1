"""Dedalus programs as Molly runs them (the fault injector whose output
faultinjectors/molly.go reads): parser and a provenance-recording evaluator.

Language (the subset the reference's case studies use, case-studies/*.ded):
  fact:  name(c1, ..., ck)@T;                       constants: "strings" or integers
  rule:  head(args)[@next|@async] :- lit, ..., lit;
         head args: Var, constant, Var+k / Var-k, count<Var>
         body: atom(args) | notin atom(args) | X op Y   (op: == != < > <= >=)
         `_` is a wildcard.
Time model (Molly's synchronous rewrite of Dedalus):
  * deductive rules run to a fixpoint inside a timestep (negation and
    aggregation stratified);
  * `@next` rules derive at t+1 on the same node and join
    clock(n, n, t, __WILDCARD__) — the node is alive at t;
  * `@async` rules send from the location of the first body atom to the
    head's first column and join clock(from, to, t, t+1): delivered at t+1
    unless the message was omitted (t < EFF) or either end has crashed;
  * crash(n, n, t) facts are visible at every timestep; a node crashed at t
    takes no clock at times >= t.
Each derived tuple records the derivations that produced it first (their body
tuples all exist before the head), so the provenance graph is acyclic.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, FrozenSet, Iterable, List, Optional, Set, Tuple

WILD = "__WILDCARD__"


# ---- syntax -------------------------------------------------------------------------
@dataclass(frozen=True)
class Var:
    name: str


@dataclass(frozen=True)
class Const:
    value: object


@dataclass(frozen=True)
class Wild:
    pass


@dataclass(frozen=True)
class Arith:
    var: str
    op: str
    k: int


@dataclass(frozen=True)
class Agg:
    fn: str
    var: str


@dataclass
class Atom:
    table: str
    args: list
    neg: bool = False


@dataclass
class Cmp:
    op: str
    left: object
    right: object


@dataclass
class Rule:
    idx: int
    head: Atom
    kind: str  # "" (deductive), "next", "async"
    body: list

    @property
    def pos(self) -> List[Atom]:
        return [b for b in self.body if isinstance(b, Atom) and not b.neg]


@dataclass
class Program:
    facts: List[Tuple[str, tuple, int]]
    rules: List[Rule]
    options: Dict[str, str] = field(default_factory=dict)


class DedalusError(ValueError):
    pass


_TOK = re.compile(r'\s+|//[^\n]*|(?P<str>"[^"]*")|(?P<num>\d+)|(?P<id>[A-Za-z_][A-Za-z0-9_]*)|'
                  r'(?P<op>:-|==|!=|<=|>=|[(),;@<>+\-])')


def _tokens(text: str) -> List[Tuple[str, str]]:
    out, i = [], 0
    while i < len(text):
        m = _TOK.match(text, i)
        if not m:
            raise DedalusError(f"unexpected {text[i]!r} at offset {i}")
        i = m.end()
        if m.lastgroup:
            out.append((m.lastgroup, m.group(m.lastgroup)))
    return out


class _P:
    def __init__(self, text: str):
        self.t = _tokens(text)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else ("eof", "")

    def eat(self, val=None, kind=None):
        tk = self.peek()
        if (val is not None and tk[1] != val) or (kind is not None and tk[0] != kind) or tk[0] == "eof":
            raise DedalusError(f"expected {val or kind}, got {tk[1]!r} (token {self.i})")
        self.i += 1
        return tk[1]

    def term(self, head: bool):
        kind, val = self.peek()
        if kind == "str":
            self.i += 1
            return Const(val[1:-1])
        if kind == "num":
            self.i += 1
            return Const(int(val))
        if kind == "id":
            self.i += 1
            if val == "_":
                return Wild()
            if head and val in ("count", "min", "max", "sum") and self.peek()[1] == "<":
                self.eat("<")
                v = self.eat(kind="id")
                self.eat(">")
                return Agg(val, v)
            if self.peek()[1] in ("+", "-"):
                op = self.eat()
                return Arith(val, op, int(self.eat(kind="num")))
            if not val[0].isupper():
                raise DedalusError(f"bad term {val!r}")
            return Var(val)
        raise DedalusError(f"bad term {val!r}")

    def atom(self, head=False, neg=False) -> Atom:
        name = self.eat(kind="id")
        self.eat("(")
        args = []
        while self.peek()[1] != ")":
            args.append(self.term(head))
            if self.peek()[1] == ",":
                self.i += 1
        self.eat(")")
        return Atom(name, args, neg)

    def literal(self):
        kind, val = self.peek()
        if kind == "id" and val == "notin":
            self.i += 1
            return self.atom(neg=True)
        if kind == "id" and self.peek(1)[1] == "(":
            return self.atom()
        left = self.term(False)
        op = self.eat()
        if op not in ("==", "!=", "<", ">", "<=", ">="):
            raise DedalusError(f"bad comparison {op!r}")
        return Cmp(op, left, self.term(False))

    def program(self) -> Program:
        facts, rules = [], []
        while self.peek()[0] != "eof":
            head = self.atom(head=True)
            kind = ""
            if self.peek()[1] == "@":
                self.i += 1
                k, v = self.peek()
                self.i += 1
                if k == "num":
                    if any(not isinstance(a, Const) for a in head.args):
                        raise DedalusError(f"fact {head.table} has non-constant arguments")
                    self.eat(";")
                    facts.append((head.table, tuple(a.value for a in head.args), int(v)))
                    continue
                if v not in ("next", "async"):
                    raise DedalusError(f"unknown temporal annotation @{v}")
                kind = v
            self.eat(":-")
            body = [self.literal()]
            while self.peek()[1] == ",":
                self.i += 1
                body.append(self.literal())
            self.eat(";")
            rules.append(Rule(len(rules), head, kind, body))
        return Program(facts, rules)


_OPT = re.compile(r"--(nodes|EOT|EFF|crashes)\s+(\S+)")


def parse(text: str) -> Program:
    """Parse a .ded program; Molly's command-line flags in its comments
    (`--nodes a,b --EOT 6 --EFF 4 --crashes 1`, case-studies/*.ded:2) become options."""
    prog = _P(text).program()
    for line in text.splitlines():
        if line.strip().startswith("//"):
            for k, v in _OPT.findall(line):
                prog.options.setdefault(k, v)
    return prog


# ---- evaluation -------------------------------------------------------------------------
Key = Tuple[str, tuple, int]  # (table, tuple, time)


@dataclass
class Derivation:
    rule: Rule
    body: Tuple[Key, ...]  # positive body goals (incl. the clock goal of next/async)


@dataclass
class FailureSpec:
    eot: int
    eff: int
    max_crashes: int
    nodes: List[str]
    crashes: Dict[str, int] = field(default_factory=dict)   # node -> crash time
    omissions: FrozenSet[Tuple[str, str, int]] = frozenset()  # (from, to, send time)

    def alive(self, n, t: int) -> bool:
        tc = self.crashes.get(n)
        return tc is None or t < tc

    def key(self):
        return (tuple(sorted(self.crashes.items())), tuple(sorted(self.omissions)))


@dataclass
class Run:
    spec: FailureSpec
    tables: Dict[int, Dict[str, Set[tuple]]]    # time -> table -> tuples
    derivs: Dict[Key, List[Derivation]]
    messages: List[Tuple[str, str, str, int, int]]  # (table, from, to, send, receive)
    success: bool = True


def _match(args, tup, env):
    env = dict(env)
    if len(args) != len(tup):
        return None
    for a, v in zip(args, tup):
        if isinstance(a, Wild):
            continue
        if isinstance(a, Const):
            if a.value != v:
                return None
        elif isinstance(a, Var):
            if a.name in env:
                if env[a.name] != v:
                    return None
            else:
                env[a.name] = v
        else:
            raise DedalusError(f"unsupported body term {a}")
    return env


def _val(term, env):
    if isinstance(term, Const):
        return term.value
    if isinstance(term, Var):
        return env[term.name]
    if isinstance(term, Arith):
        v = env[term.var]
        return v + term.k if term.op == "+" else v - term.k
    raise DedalusError(f"cannot evaluate {term}")


_CMP = {"==": lambda a, b: a == b, "!=": lambda a, b: a != b, "<": lambda a, b: a < b, ">": lambda a, b: a > b,
        "<=": lambda a, b: a <= b, ">=": lambda a, b: a >= b}


def _bindings(rule: Rule, db: Dict[str, Set[tuple]], t: int):
    """Every satisfying binding of the body with its positive body keys."""
    pos = rule.pos
    out = []

    def rec(i, env, used):
        if i == len(pos):
            for b in rule.body:
                if isinstance(b, Atom) and b.neg:
                    if any(_match(b.args, tup, env) is not None for tup in db.get(b.table, ())):
                        return
                elif isinstance(b, Cmp):
                    try:
                        if not _CMP[b.op](_val(b.left, env), _val(b.right, env)):
                            return
                    except TypeError:
                        return
            out.append((env, tuple(used)))
            return
        a = pos[i]
        for tup in sorted(db.get(a.table, ()), key=repr):
            e = _match(a.args, tup, env)
            if e is not None:
                rec(i + 1, e, used + [(a.table, tup, t)])

    rec(0, {}, [])
    return out


def _heads(rule: Rule, binds):
    """(head tuple, body keys) per binding; aggregates group over the other head columns."""
    h = rule.head
    aggs = [i for i, a in enumerate(h.args) if isinstance(a, Agg)]
    if not aggs:
        return [(tuple(_val(a, env) for a in h.args), used) for env, used in binds]
    groups: Dict[tuple, Tuple[set, list]] = {}
    for env, used in binds:
        g = tuple(_val(a, env) if not isinstance(a, Agg) else None for a in h.args)
        vals, bodies = groups.setdefault(g, (set(), []))
        vals.add(env[h.args[aggs[0]].var])
        bodies.extend(u for u in used if u not in bodies)
    out = []
    for g, (vals, bodies) in groups.items():
        fn = h.args[aggs[0]].fn
        v = len(vals) if fn == "count" else min(vals) if fn == "min" else max(vals) if fn == "max" else sum(vals)
        out.append((tuple(v if isinstance(a, Agg) else g[i] for i, a in enumerate(h.args)), tuple(bodies)))
    return out


def _strata(rules: List[Rule]) -> List[List[Rule]]:
    ded = [r for r in rules if r.kind == ""]
    level: Dict[str, int] = {r.head.table: 0 for r in ded}
    for _ in range(len(ded) + 2):
        changed = False
        for r in ded:
            agg = any(isinstance(a, Agg) for a in r.head.args)
            for b in r.body:
                if isinstance(b, Atom) and b.table in level:
                    need = level[b.table] + (1 if (b.neg or agg) else 0)
                    if need > level[r.head.table]:
                        level[r.head.table] = need
                        changed = True
        if not changed:
            break
    else:
        raise DedalusError("program is not stratifiable (recursion through negation or aggregation)")
    n = max(level.values(), default=-1) + 1
    return [[r for r in ded if level[r.head.table] == s] for s in range(n)]


def evaluate(prog: Program, spec: FailureSpec) -> Run:
    strata = _strata(prog.rules)
    carry = [r for r in prog.rules if r.kind in ("next", "async")]
    tables: Dict[int, Dict[str, Set[tuple]]] = {}
    derivs: Dict[Key, List[Derivation]] = {}
    messages = []
    pending: Dict[str, Set[tuple]] = {}
    pending_d: Dict[Key, List[Derivation]] = {}
    for t in range(1, spec.eot + 1):
        db: Dict[str, Set[tuple]] = {}
        for tab, tup, ft in prog.facts:
            if ft == t:
                db.setdefault(tab, set()).add(tup)
        for n, tc in spec.crashes.items():
            db.setdefault("crash", set()).add((n, n, tc))
        for tab, tups in pending.items():
            db.setdefault(tab, set()).update(tups)
        for k, ds in pending_d.items():
            derivs.setdefault(k, []).extend(ds)
        pending, pending_d = {}, {}
        for stratum in strata:
            while True:
                new = []
                for r in stratum:
                    for head, used in _heads(r, _bindings(r, db, t)):
                        if head not in db.get(r.head.table, ()):
                            new.append((r, head, used))
                if not new:
                    break
                for r, head, used in new:
                    key = (r.head.table, head, t)
                    if head not in db.get(r.head.table, ()):
                        db.setdefault(r.head.table, set()).add(head)
                    ds = derivs.setdefault(key, [])
                    if all(d.body != used or d.rule.idx != r.idx for d in ds):
                        ds.append(Derivation(r, used))
        tables[t] = db
        if t == spec.eot:
            break
        for r in carry:
            for head, used in _heads(r, _bindings(r, db, t)):
                if r.kind == "next":
                    loc = head[0]
                    if not spec.alive(loc, t):
                        continue
                    clock = ("clock", (loc, loc, t, WILD), t)
                else:
                    loc = used[0][1][0] if used else head[0]
                    dest = head[0]
                    if not (spec.alive(loc, t) and spec.alive(dest, t + 1)):
                        continue
                    if loc != dest and t < spec.eff and (loc, dest, t) in spec.omissions:
                        continue
                    clock = ("clock", (loc, dest, t, t + 1), t)
                    messages.append((r.head.table, loc, dest, t, t + 1))
                key = (r.head.table, head, t + 1)
                pending.setdefault(r.head.table, set()).add(head)
                ds = pending_d.setdefault(key, [])
                body = tuple(used) + (clock,)
                if all(d.body != body or d.rule.idx != r.idx for d in ds):
                    ds.append(Derivation(r, body))
    last = tables[spec.eot]
    pre, post = last.get("pre", set()), last.get("post", set())
    return Run(spec, tables, derivs, sorted(set(messages)), success=pre <= post)


def goals_of(run: Run, table: str) -> List[Key]:
    """Every (table, tuple, t) instance in the model, by time."""
    return [(table, tup, t) for t in sorted(run.tables) for tup in sorted(run.tables[t].get(table, ()), key=repr)]


def label(key: Key) -> str:
    tab, tup, _ = key
    return f"{tab}({', '.join(str(v) for v in tup)})"


def reachable(run: Run, roots: Iterable[Key]) -> Tuple[List[Key], List[Tuple[Key, Derivation]]]:
    """Goals and (head, derivation) rule instances reachable from `roots`, in DFS order."""
    seen: Set[Key] = set()
    goals: List[Key] = []
    rules: List[Tuple[Key, Derivation]] = []
    stack = list(reversed(list(roots)))
    while stack:
        k = stack.pop()
        if k in seen:
            continue
        seen.add(k)
        goals.append(k)
        for d in run.derivs.get(k, []):
            rules.append((k, d))
            for b in reversed(d.body):
                if b not in seen:
                    stack.append(b)
    return goals, rules
