"""Safe, vectorized evaluator for the JEXL subset Shifu uses in ``filterExpressions``,
``weightColumnName`` expressions and segment files (replaces commons-jexl2 in
``DataPurifier.isFilter`` J/core/DataPurifier.java:103-145; syntax covered by
``src/test/java/ml/shifu/shifu/util/JexlTest.java``).

Supported: numbers, 'str'/"str", null/true/false, column identifiers (incl. ``ns::name``),
``== != < <= > >= eq ne lt le gt ge``, ``&& || ! and or not``, ``+ - * / %``, parentheses,
methods ``.isEmpty() .equals(x) .substring(a[,b]) .startsWith(x) .endsWith(x) .contains(x)
.length() .trim() .toLowerCase() .toUpperCase()``, ``NumberUtils.max/min(...)``,
``Math.abs/log/exp/sqrt/pow/max/min(...)``.  Evaluation is column-at-a-time over numpy arrays;
nothing is ``eval``'d.
"""
from __future__ import annotations

import re

import numpy as np

_TOK = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[dDfFlL]?)
  | (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<op>==|!=|<=|>=|&&|\|\||=~|[<>!+\-*/%(),.])
  | (?P<id>[A-Za-z_$][A-Za-z0-9_$]*(?:::[A-Za-z0-9_$]+)*)
""", re.X)

_KW = {"and": "&&", "or": "||", "not": "!", "eq": "==", "ne": "!=", "lt": "<", "le": "<=", "gt": ">",
       "ge": ">="}


class ExprError(ValueError):
    pass


def tokenize(s: str):
    pos, out = 0, []
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m:
            raise ExprError(f"bad token at {pos}: {s[pos:pos + 10]!r}")
        pos = m.end()
        kind = m.lastgroup
        v = m.group()
        if kind == "ws":
            continue
        if kind == "id" and v.lower() in _KW:
            out.append(("op", _KW[v.lower()]))
        elif kind == "id" and v in ("null", "true", "false"):
            out.append(("lit", {"null": None, "true": True, "false": False}[v]))
        elif kind == "num":
            out.append(("lit", float(v.rstrip("dDfFlL"))))
        elif kind == "str":
            out.append(("lit", bytes(v[1:-1], "utf-8").decode("unicode_escape")))
        else:
            out.append((kind, v))
    out.append(("eof", None))
    return out


_BP = {"||": 1, "&&": 2, "==": 3, "!=": 3, "=~": 3, "<": 4, "<=": 4, ">": 4, ">=": 4, "+": 5, "-": 5,
       "*": 6, "/": 6, "%": 6}


class Parser:
    def __init__(self, s):
        self.t = tokenize(s)
        self.i = 0

    def peek(self):
        return self.t[self.i]

    def next(self):
        tk = self.t[self.i]
        self.i += 1
        return tk

    def expect(self, v):
        tk = self.next()
        if tk[1] != v:
            raise ExprError(f"expected {v!r}, got {tk[1]!r}")

    def parse(self):
        e = self.expr(0)
        if self.peek()[0] != "eof":
            raise ExprError(f"trailing tokens from {self.peek()}")
        return e

    def expr(self, rbp):
        left = self.nud()
        while True:
            tk = self.peek()
            if tk[0] == "op" and tk[1] in _BP and _BP[tk[1]] > rbp:
                self.next()
                right = self.expr(_BP[tk[1]])
                left = ("bin", tk[1], left, right)
            elif tk[0] == "op" and tk[1] == ".":
                self.next()
                name = self.next()
                if name[0] != "id":
                    raise ExprError("method name expected")
                args = self.args()
                left = ("call", name[1], left, args)
            else:
                return left

    def args(self):
        self.expect("(")
        args = []
        if self.peek()[1] != ")":
            while True:
                args.append(self.expr(0))
                if self.peek()[1] == ",":
                    self.next()
                    continue
                break
        self.expect(")")
        return args

    def nud(self):
        tk = self.next()
        if tk[0] == "lit":
            return ("lit", tk[1])
        if tk[0] == "op" and tk[1] == "(":
            e = self.expr(0)
            self.expect(")")
            return e
        if tk[0] == "op" and tk[1] in ("!", "-", "+"):
            e = self.expr(7)
            return ("un", tk[1], e)
        if tk[0] == "id":
            if tk[1] in ("NumberUtils", "Math") and self.peek()[1] == ".":
                self.next()
                fn = self.next()[1]
                return ("fn", f"{tk[1]}.{fn}", self.args())
            if tk[1] in ("empty", "size") and self.peek()[1] == "(":
                return ("fn", tk[1], self.args())
            return ("col", tk[1])
        raise ExprError(f"unexpected token {tk}")


class Vec:
    """A column or computed vector with lazy numeric / string views."""

    def __init__(self, num=None, strs=None, missing=None):
        self._num = num
        self._str = strs
        self._miss = missing

    @staticmethod
    def of_column(col):
        return Vec(None, None, None) if col is None else _ColVec(col)

    def num(self):
        if self._num is None:
            s = self.str()
            out = np.full(len(s), np.nan)
            for i, v in enumerate(s):
                try:
                    out[i] = float(v) if v not in ("", None) else np.nan
                except (TypeError, ValueError):
                    pass
            self._num = out
        return self._num

    def str(self):
        if self._str is None:
            n = self._num
            self._str = np.array(["" if v != v else (repr(float(v))) for v in n], dtype=object)
        return self._str

    def missing(self):
        if self._miss is None:
            if self._str is not None:
                self._miss = np.array([v is None or v == "" for v in self._str])
            else:
                self._miss = np.isnan(self._num)
        return self._miss

    def __len__(self):
        return len(self._num) if self._num is not None else len(self.str())


class _ColVec(Vec):
    def __init__(self, col):
        super().__init__()
        self.col = col

    def num(self):
        if self._num is None:
            self._num = self.col.numeric()
        return self._num

    def str(self):
        if self._str is None:
            self._str = self.col.strings()
        return self._str

    def missing(self):
        if self._miss is None:
            self._miss = self.col.missing_mask()
        return self._miss

    def __len__(self):
        return len(self.col.values)


def _as_num(x, n):
    if isinstance(x, Vec):
        return x.num()
    if isinstance(x, np.ndarray):
        return x.astype(np.float64) if x.dtype != object else Vec(strs=x).num()
    if x is None:
        return np.full(n, np.nan)
    if isinstance(x, bool):
        return np.full(n, float(x))
    if isinstance(x, str):
        try:
            return np.full(n, float(x))
        except ValueError:
            return np.full(n, np.nan)
    return np.full(n, float(x))


def _as_str(x, n):
    if isinstance(x, Vec):
        return x.str()
    if isinstance(x, np.ndarray):
        if x.dtype == object:
            return x
        return Vec(num=x.astype(float)).str()
    if x is None:
        return np.array([None] * n, dtype=object)
    return np.array([x if isinstance(x, str) else repr(x)] * n, dtype=object)


def _as_bool(x, n):
    if isinstance(x, np.ndarray) and x.dtype == bool:
        return x
    if isinstance(x, bool):
        return np.full(n, x)
    if isinstance(x, Vec):
        s = x.str()
        return np.array([str(v).lower() == "true" for v in s])
    if isinstance(x, np.ndarray):
        return x.astype(bool)
    return np.full(n, bool(x))


def _is_numeric_like(x):
    if isinstance(x, (int, float)) and not isinstance(x, bool):
        return True
    if isinstance(x, np.ndarray) and x.dtype != object and x.dtype != bool:
        return True
    if isinstance(x, _ColVec) and x.col.kind == "num":
        return True
    if isinstance(x, Vec) and not isinstance(x, _ColVec) and x._num is not None and x._str is None:
        return True
    return False


class Evaluator:
    def __init__(self, expr: str):
        self.expr = expr
        self.ast = Parser(expr).parse()

    def columns(self):
        out = []

        def walk(a):
            if a[0] == "col":
                out.append(a[1])
            elif a[0] in ("bin",):
                walk(a[2]); walk(a[3])
            elif a[0] == "un":
                walk(a[2])
            elif a[0] == "call":
                walk(a[2])
                for x in a[3]:
                    walk(x)
            elif a[0] == "fn":
                for x in a[2]:
                    walk(x)
        walk(self.ast)
        return out

    def eval(self, table, n=None):
        from ..config.updater import simple_name
        self.n = table.n if n is None else n
        self.table = table
        self._simple = {simple_name(k): k for k in table.columns}
        return self._ev(self.ast)

    def mask(self, table):
        v = self.eval(table)
        return _as_bool(v, table.n)

    def values(self, table):
        return _as_num(self.eval(table), table.n)

    def _ev(self, a):
        n = self.n
        k = a[0]
        if k == "lit":
            return a[1]
        if k == "col":
            name = a[1]
            col = self.table.columns.get(name)
            if col is None:
                from ..config.updater import simple_name
                alt = self._simple.get(simple_name(name))
                col = self.table.columns.get(alt) if alt else None
            if col is None:
                return None    # unknown variable -> null (JEXL lenient)
            return _ColVec(col)
        if k == "un":
            v = self._ev(a[2])
            if a[1] == "!":
                return ~_as_bool(v, n)
            if a[1] == "-":
                return -_as_num(v, n)
            return _as_num(v, n)
        if k == "bin":
            op, l, r = a[1], self._ev(a[2]), self._ev(a[3])
            if op == "&&":
                return _as_bool(l, n) & _as_bool(r, n)
            if op == "||":
                return _as_bool(l, n) | _as_bool(r, n)
            if op in ("==", "!="):
                if l is None or r is None:
                    other = r if l is None else l
                    if other is None:
                        res = np.full(n, True)
                    elif isinstance(other, Vec):
                        res = other.missing()
                    else:
                        res = np.full(n, False)
                    return res if op == "==" else ~res
                if _is_numeric_like(l) or _is_numeric_like(r):
                    ln, rn = _as_num(l, n), _as_num(r, n)
                    with np.errstate(invalid="ignore"):
                        res = ln == rn
                    # string literal that is not a number compared with a number column
                    if isinstance(l, str) or isinstance(r, str):
                        lit = l if isinstance(l, str) else r
                        try:
                            float(lit)
                        except ValueError:
                            res = _as_str(l, n) == _as_str(r, n)
                else:
                    res = _as_str(l, n) == _as_str(r, n)
                res = np.asarray(res, dtype=bool)
                return res if op == "==" else ~res
            if op == "=~":
                rx = re.compile(str(r))
                return np.array([bool(rx.fullmatch(str(s))) for s in _as_str(l, n)])
            if op in ("<", "<=", ">", ">="):
                ln, rn = _as_num(l, n), _as_num(r, n)
                with np.errstate(invalid="ignore"):
                    return {"<": ln < rn, "<=": ln <= rn, ">": ln > rn, ">=": ln >= rn}[op]
            ln, rn = _as_num(l, n), _as_num(r, n)
            if op == "+":
                if isinstance(l, str) or isinstance(r, str) or (
                        isinstance(l, Vec) and not _is_numeric_like(l) and np.isnan(ln).all()):
                    return np.array([f"{x}{y}" for x, y in zip(_as_str(l, n), _as_str(r, n))], dtype=object)
                return ln + rn
            with np.errstate(divide="ignore", invalid="ignore"):
                if op == "-":
                    return ln - rn
                if op == "*":
                    return ln * rn
                if op == "/":
                    return ln / rn
                if op == "%":
                    return np.fmod(ln, rn)
            raise ExprError(op)
        if k == "call":
            name, obj, args = a[1], self._ev(a[2]), [self._ev(x) for x in a[3]]
            s = _as_str(obj, n)
            if name == "isEmpty":
                return np.array([v is None or v == "" for v in s])
            if name == "equals":
                return s == _as_str(args[0], n)
            if name == "equalsIgnoreCase":
                t = _as_str(args[0], n)
                return np.array([str(x).lower() == str(y).lower() for x, y in zip(s, t)])
            if name == "length":
                return np.array([len(v or "") for v in s], dtype=float)
            if name == "trim":
                return np.array([(v or "").strip() for v in s], dtype=object)
            if name == "toLowerCase":
                return np.array([(v or "").lower() for v in s], dtype=object)
            if name == "toUpperCase":
                return np.array([(v or "").upper() for v in s], dtype=object)
            if name == "substring":
                b = int(_as_num(args[0], 1)[0])
                e = int(_as_num(args[1], 1)[0]) if len(args) > 1 else None
                return np.array([(v or "")[b:e] for v in s], dtype=object)
            if name in ("startsWith", "endsWith", "contains"):
                t = _as_str(args[0], n)
                f = {"startsWith": str.startswith, "endsWith": str.endswith,
                     "contains": lambda x, y: y in x}[name]
                return np.array([f(str(x or ""), str(y or "")) for x, y in zip(s, t)])
            raise ExprError(f"unsupported method {name}")
        if k == "fn":
            name, args = a[1], [self._ev(x) for x in a[2]]
            if name in ("NumberUtils.max", "Math.max"):
                return np.nanmax(np.stack([_as_num(x, n) for x in args]), axis=0)
            if name in ("NumberUtils.min", "Math.min"):
                return np.nanmin(np.stack([_as_num(x, n) for x in args]), axis=0)
            one = {"Math.abs": np.abs, "Math.log": np.log, "Math.exp": np.exp, "Math.sqrt": np.sqrt,
                   "Math.log10": np.log10, "Math.floor": np.floor, "Math.ceil": np.ceil}
            if name in one:
                with np.errstate(divide="ignore", invalid="ignore"):
                    return one[name](_as_num(args[0], n))
            if name == "Math.pow":
                return np.power(_as_num(args[0], n), _as_num(args[1], n))
            if name == "empty":
                v = args[0]
                return v.missing() if isinstance(v, Vec) else np.full(n, v is None or v == "")
            if name == "size":
                return np.array([len(v or "") for v in _as_str(args[0], n)], dtype=float)
            raise ExprError(f"unsupported function {name}")
        raise ExprError(f"bad node {a}")


def compile_expr(expr: str) -> Evaluator:
    return Evaluator(expr)
