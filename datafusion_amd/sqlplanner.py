"""Host SQL front end (unchanged semantics of src/sqlplanner.rs:45-359 +
sqlparser 0.1.8 precedence): ``SELECT <expr>, ... [FROM <table>] [WHERE
<expr>] [GROUP BY <expr>, ...] [ORDER BY <expr> [ASC|DESC], ...] [LIMIT n]``
-> Limit?(Sort?(Projection(Selection?(TableScan | EmptyRelation)))) or
Aggregate(Selection?(TableScan)); the plans' Debug strings are pinned to the
reference's planner tests (tests/test_planner_debug_cpu.py).

Literal typing (sqlplanner.rs:204-212): integer -> Int64, decimal -> Float64,
quoted -> Utf8. Binary operators cast both sides to their supertype
(sqlplanner.rs:272-287), which is where the executable Cast(Literal) nodes
and the non-executable Cast(Column) nodes come from.
"""
from __future__ import annotations

import re
from typing import List

from .logicalplan import (AggregateFunction, BinaryExpr, Cast, Column, DataType, Float64, Int64, IsNotNull, IsNull,
                          Literal, Operator, PlanError, ScalarFunction, SortExpr, Utf8, binary_expr_coerced)

_TOKEN = re.compile(r"""\s*(?:(?P<num>\d+\.\d*|\.\d+|\d+)|(?P<str>'(?:[^']|'')*')|(?P<op><>|!=|<=|>=|[=<>+\-*/%(),])|(?P<id>[A-Za-z_][A-Za-z0-9_]*))""")

_PREC = {"OR": 5, "AND": 10, "=": 20, "!=": 20, "<>": 20, "<": 20, "<=": 20, ">": 20, ">=": 20,
         "+": 30, "-": 30, "*": 40, "/": 40, "%": 40}
_OPS = {"=": Operator.Eq, "!=": Operator.NotEq, "<>": Operator.NotEq, "<": Operator.Lt, "<=": Operator.LtEq,
        ">": Operator.Gt, ">=": Operator.GtEq, "+": Operator.Plus, "-": Operator.Minus,
        "*": Operator.Multiply, "/": Operator.Divide, "%": Operator.Modulus, "AND": Operator.And,
        "OR": Operator.Or}
_TYPES = {"BOOLEAN": DataType.Boolean, "SMALLINT": DataType.Int16, "INT": DataType.Int32,
          "INTEGER": DataType.Int32, "BIGINT": DataType.Int64, "FLOAT": DataType.Float64,
          "REAL": DataType.Float64, "DOUBLE": DataType.Float64, "VARCHAR": DataType.Utf8,
          "CHAR": DataType.Utf8}


def tokenize(sql: str) -> List[tuple]:
    out, pos = [], 0
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            if sql[pos:].strip() == "":
                break
            raise PlanError("Unexpected character at %d in %r" % (pos, sql))
        pos = m.end()
        if m.group("num"):
            out.append(("num", m.group("num")))
        elif m.group("str"):
            out.append(("str", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("op"):
            out.append(("op", m.group("op")))
        else:
            w = m.group("id")
            out.append(("kw", w.upper()) if w.upper() in ("SELECT", "FROM", "WHERE", "AND", "OR", "CAST", "AS",
                                                          "IS", "NOT", "NULL") else ("id", w))
    return out


class SqlToRel:
    def __init__(self, ctx):
        self.ctx = ctx

    def sql_to_rel(self, sql: str):
        """sqlplanner.rs:45-180: the input relation (FROM, else EmptyRelation),
        Selection, then Aggregate (when the projection holds an aggregate) or
        Projection -> Sort (ORDER BY, resolved against the projection's
        schema) -> Limit."""
        from .arrow import Schema
        from .execution.context import (Aggregate, EmptyRelation, Limit, Projection, Selection, Sort, TableScan,
                                        exprlist_to_fields)
        self.toks = tokenize(sql)
        self.i = 0
        self._expect("kw", "SELECT")
        proj_src = []
        while True:
            start = self.i
            self._skip_expr()
            proj_src.append((start, self.i))
            if self._peek() == ("op", ","):
                self.i += 1
                continue
            break
        if self._peek() == ("kw", "FROM"):
            self.i += 1
            t = self._next()
            if t[0] != "id":
                raise PlanError("expected table name")
            table = t[1]
            schema = self.ctx.table_schema(table)
            if schema is None:
                raise PlanError("no schema found for table %s" % table)
            plan = TableScan(table, schema)
        else:  # sqlplanner.rs:58-63
            schema = Schema([])
            plan = EmptyRelation(schema)
        where = None
        if self._peek() == ("kw", "WHERE"):
            self.i += 1
            where = self._parse_expr(0, schema)
        group_src = None
        if self._peek_id("GROUP"):
            self.i += 1
            if not self._peek_id("BY"):
                raise PlanError("expected BY")
            self.i += 1
            group_src = []
            while True:
                group_src.append(self._parse_expr(0, schema))
                if self._peek() != ("op", ","):
                    break
                self.i += 1
        order_src = []  # (token range, asc)
        if self._peek_id("ORDER"):
            self.i += 1
            if not self._peek_id("BY"):
                raise PlanError("expected BY")
            self.i += 1
            while True:
                a = self.i
                self._skip_order_key()
                b = self.i
                asc = True
                if self._peek_id("ASC") or self._peek_id("DESC"):
                    asc = self._next()[1].upper() == "ASC"
                order_src.append((a, b, asc))
                if self._peek() != ("op", ","):
                    break
                self.i += 1
        limit = None
        if self._peek_id("LIMIT"):
            self.i += 1
            t = self._next()
            if t[0] != "num" or "." in t[1]:
                raise PlanError("LIMIT parameter is not a number")
            limit = int(t[1])
        if self.i != len(self.toks):
            raise PlanError("unexpected token %r" % (self.toks[self.i],))
        end = self.i
        exprs = []
        for (a, b) in proj_src:
            self.i = a
            if self.toks[a] == ("op", "*"):
                raise PlanError("SQL wildcard operator is not supported in projection - please use explicit column names")
            exprs.append(self._parse_expr(0, schema))
            if self.i != b:
                raise PlanError("bad projection expression")
        self.i = end
        if where is not None:
            plan = Selection(where, plan)
        aggr = [e for e in exprs if isinstance(e, AggregateFunction)]
        if aggr:  # sqlplanner.rs:80-117: only the aggregate expressions are kept
            return Aggregate(plan, group_src or [], aggr)
        proj_schema = Schema(exprlist_to_fields(exprs, schema))
        plan = Projection(exprs, plan, proj_schema)
        if order_src:  # sqlplanner.rs:139-161
            keys = []
            for a, b, asc in order_src:
                self.i = a
                keys.append(SortExpr(self._parse_expr(0, proj_schema), asc))
                if self.i != b:
                    raise PlanError("bad ORDER BY expression")
            plan = Sort(keys, plan, proj_schema)
        if limit is not None:  # sqlplanner.rs:163-176
            plan = Limit(limit, plan, proj_schema)
        self.i = end
        return plan

    # -- helpers
    def _peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else (None, None)

    def _next(self):
        t = self._peek()
        self.i += 1
        return t

    def _expect(self, kind, val):
        t = self._next()
        if t != (kind, val):
            raise PlanError("expected %s, got %r" % (val, t))

    def _peek_id(self, word):
        t = self._peek()
        return t[0] == "id" and t[1].upper() == word

    def _skip_order_key(self):
        depth = 0
        while self.i < len(self.toks):
            t = self.toks[self.i]
            if t == ("op", "("):
                depth += 1
            elif t == ("op", ")"):
                depth -= 1
            elif depth == 0 and (t == ("op", ",") or (t[0] == "id" and t[1].upper() in ("ASC", "DESC", "LIMIT"))):
                return
            self.i += 1

    def _skip_expr(self):
        depth = 0
        while self.i < len(self.toks):
            t = self.toks[self.i]
            if t == ("op", "("):
                depth += 1
            elif t == ("op", ")"):
                depth -= 1
            elif depth == 0 and (t == ("op", ",") or t == ("kw", "FROM")):
                return
            self.i += 1

    def _binop(self):
        t = self._peek()
        if t[0] == "op" and t[1] in _PREC:
            return t[1]
        if t[0] == "kw" and t[1] in ("AND", "OR"):
            return t[1]
        return None

    def _parse_expr(self, min_prec, schema):
        left = self._parse_prefix(schema)
        while True:
            op = self._binop()
            if op is None:
                if self._peek() == ("kw", "IS"):
                    self.i += 1
                    neg = self._peek() == ("kw", "NOT")
                    if neg:
                        self.i += 1
                    self._expect("kw", "NULL")
                    left = IsNotNull(left) if neg else IsNull(left)
                    continue
                return left
            prec = _PREC[op]
            if prec <= min_prec:
                return left
            self.i += 1
            right = self._parse_expr(prec, schema)
            left = binary_expr_coerced(left, _OPS[op], right, schema)

    def _parse_prefix(self, schema):
        t = self._next()
        if t[0] == "num":
            return Literal(Float64(float(t[1]))) if "." in t[1] else Literal(Int64(int(t[1])))
        if t[0] == "str":
            return Literal(Utf8(t[1]))
        if t == ("op", "-"):
            n = self._next()
            if n[0] != "num":
                raise PlanError("unsupported unary minus")
            return Literal(Float64(-float(n[1]))) if "." in n[1] else Literal(Int64(-int(n[1])))
        if t == ("op", "("):
            e = self._parse_expr(0, schema)
            self._expect("op", ")")
            return e
        if t == ("kw", "CAST"):
            self._expect("op", "(")
            e = self._parse_expr(0, schema)
            self._expect("kw", "AS")
            ty = self._next()
            if ty[0] not in ("id", "kw") or ty[1].upper() not in _TYPES:
                raise PlanError("unsupported type %r" % (ty,))
            if self._peek() == ("op", "("):  # VARCHAR(100)
                self.i += 3
            self._expect("op", ")")
            return Cast(e, _TYPES[ty[1].upper()])
        if t[0] == "id" and self._peek() == ("op", "("):  # SQLFunction (sqlplanner.rs:292-330)
            return self._parse_function(t[1], schema)
        if t[0] == "id":
            for i, f in enumerate(schema.fields):
                if f.name == t[1]:
                    return Column(i)
            raise PlanError("Invalid identifier '%s' for schema %s" % (t[1], schema.to_string()))
        raise PlanError("Unsupported ast node %r in sqltorel" % (t,))

    def _parse_function(self, name, schema):
        self._expect("op", "(")
        lname = name.lower()
        args = []
        while self._peek() != ("op", ")"):
            if lname == "count" and self._peek() in (("op", "*"), ("num", "1")):
                self.i += 1  # COUNT(*) / COUNT(1) -> COUNT(first column)
                args.append(Column(0))
            else:
                args.append(self._parse_expr(0, schema))
            if self._peek() == ("op", ","):
                self.i += 1
        self._expect("op", ")")
        if lname in ("min", "max", "sum", "avg"):
            # return type is the argument's type (sqlplanner.rs:301-303)
            return AggregateFunction(name, tuple(args), args[0].get_type(schema))
        if lname == "count":
            return AggregateFunction(name, tuple(args), DataType.UInt64)
        # a scalar function of the schema provider: each argument cast to the
        # declared parameter type (sqlplanner.rs:330-350)
        meta = getattr(self.ctx, "function_meta", None)
        fm = meta(name) if meta is not None else None
        if fm is None:
            raise PlanError("Invalid function '%s'" % name)
        arg_types, return_type = fm
        return ScalarFunction(name, tuple(a.cast_to(t, schema) for a, t in zip(args, arg_types)), return_type)
