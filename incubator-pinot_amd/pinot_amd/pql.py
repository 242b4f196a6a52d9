"""PQL subset compiler: the query text -> the BrokerRequest pieces the server hot path reads.

Restates the predicate compilation of pinot-common's PQL2 front end
(`pinot-common/src/main/java/org/apache/pinot/pql/parsers/pql2/ast/`):
  * `=`      -> EQUALITY [v]                               ComparisonPredicateAstNode.java:133-139
  * `<>`/`!=`-> NOT [v]                                    :140-146
  * `<`      -> RANGE "(*\\t\\tv)";  `<=` -> "(*\\t\\tv]"   :99-110  (identifier on the left)
  * `>`      -> RANGE "(v\\t\\t*)";  `>=` -> "[v\\t\\t*)"   :111-122
  * BETWEEN  -> RANGE "[a\\t\\tb]"                          BetweenPredicateAstNode.java:76
  * IN / NOT IN -> IN / NOT_IN with the values joined by "\\t\\t"   InPredicateAstNode.java:106-170
  * AND/OR chains are flattened into one n-ary node.
Literal text follows `LiteralAstNode.getValueAsString` (integers as Long.toString, strings unquoted).
Supported statement: SELECT agg(col|*)[, ...] FROM t [WHERE ...] [GROUP BY c[, ...]] [TOP n] [LIMIT n].
"""
import re

AGG_FUNCTIONS = ("COUNT", "SUM", "MIN", "MAX", "AVG", "DISTINCTCOUNTHLL", "COUNTMV", "SUMMV", "MINMV", "MAXMV", "AVGMV",
                 "DISTINCTCOUNTHLLMV")
_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+\.\d*(?:[eE][-+]?\d+)?|-?\d+(?:[eE][-+]?\d+)?)|"
                    r"(?P<str>'(?:[^']|'')*'|\"(?:[^\"]|\"\")*\")|"
                    r"(?P<op><>|!=|<=|>=|=|<|>|\(|\)|,|\*)|(?P<id>[A-Za-z_][A-Za-z0-9_.$]*))")
_KEYWORDS = {"SELECT", "FROM", "WHERE", "AND", "OR", "NOT", "IN", "BETWEEN", "GROUP", "BY", "TOP", "LIMIT"}


class PqlCompilationException(ValueError):
    pass


def _tokenize(text):
    pos = 0
    out = []
    text = text.strip()
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            raise PqlCompilationException("cannot parse near: %r" % text[pos:pos + 20])
        pos = m.end()
        if m.group("num") is not None:
            out.append(("lit", _number_text(m.group("num"))))
        elif m.group("str") is not None:
            s = m.group("str")
            q = s[0]
            out.append(("lit", s[1:-1].replace(q + q, q)))
        elif m.group("op") is not None:
            out.append(("op", m.group("op")))
        else:
            word = m.group("id")
            out.append(("kw", word.upper()) if word.upper() in _KEYWORDS else ("id", word))
    return out


def _number_text(s):
    if re.fullmatch(r"-?\d+", s):
        return str(int(s))  # IntegerLiteralAstNode: Long.toString
    v = float(s)
    r = repr(v)
    return r  # FloatingPointLiteralAstNode: Double.toString (matches for plain decimals)


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, kind=None, val=None):
        tok = self.peek()
        if tok[0] is None or (kind and tok[0] != kind) or (val and tok[1] != val):
            raise PqlCompilationException("expected %s %s, got %r" % (kind, val, tok))
        self.i += 1
        return tok

    def accept(self, kind, val=None):
        tok = self.peek()
        if tok[0] == kind and (val is None or tok[1] == val):
            self.i += 1
            return True
        return False

    def query(self):
        self.take("kw", "SELECT")
        aggs = [self.agg()]
        while self.accept("op", ","):
            aggs.append(self.agg())
        self.take("kw", "FROM")
        table = self.take("id")[1]
        flt = None
        group = None
        top = None
        if self.accept("kw", "WHERE"):
            flt = self.or_expr()
        if self.accept("kw", "GROUP"):
            self.take("kw", "BY")
            cols = [self.take("id")[1]]
            while self.accept("op", ","):
                cols.append(self.take("id")[1])
            group = cols
        while self.peek()[0] == "kw" and self.peek()[1] in ("TOP", "LIMIT"):
            kw = self.take("kw")[1]
            n = int(self.take("lit")[1])
            if kw == "TOP":
                top = n
        if self.peek()[0] is not None:
            raise PqlCompilationException("trailing tokens: %r" % (self.t[self.i:],))
        q = {"table": table, "aggregations": aggs, "filter": flt, "group_by": None}
        if group:
            q["group_by"] = {"columns": group, "top_n": top if top is not None else 10}
        return q

    def agg(self):
        fn = self.take("id")[1].upper()
        if fn not in AGG_FUNCTIONS:
            raise PqlCompilationException("unsupported aggregation function %s" % fn)
        self.take("op", "(")
        if self.accept("op", "*"):
            col = "*"
        else:
            col = self.take("id")[1]
        self.take("op", ")")
        return {"function": fn, "column": col}

    def or_expr(self):
        kids = [self.and_expr()]
        while self.accept("kw", "OR"):
            kids.append(self.and_expr())
        return kids[0] if len(kids) == 1 else _flatten("OR", kids)

    def and_expr(self):
        kids = [self.pred()]
        while self.accept("kw", "AND"):
            kids.append(self.pred())
        return kids[0] if len(kids) == 1 else _flatten("AND", kids)

    def pred(self):
        if self.accept("op", "("):
            e = self.or_expr()
            self.take("op", ")")
            return e
        col = self.take("id")[1]
        tok = self.peek()
        if tok == ("kw", "BETWEEN"):
            self.i += 1
            a = self.take("lit")[1]
            self.take("kw", "AND")
            b = self.take("lit")[1]
            return {"operator": "RANGE", "column": col, "values": ["[%s\t\t%s]" % (a, b)]}
        negate = False
        if tok == ("kw", "NOT"):
            self.i += 1
            negate = True
        if self.accept("kw", "IN"):
            self.take("op", "(")
            vals = [self.take("lit")[1]]
            while self.accept("op", ","):
                vals.append(self.take("lit")[1])
            self.take("op", ")")
            return {"operator": "NOT_IN" if negate else "IN", "column": col, "values": ["\t\t".join(vals)]}
        if negate:
            raise PqlCompilationException("NOT must be followed by IN")
        op = self.take("op")[1]
        v = self.take("lit")[1]
        if op == "=":
            return {"operator": "EQUALITY", "column": col, "values": [v]}
        if op in ("<>", "!="):
            return {"operator": "NOT", "column": col, "values": [v]}
        rng = {"<": "(*\t\t%s)", "<=": "(*\t\t%s]", ">": "(%s\t\t*)", ">=": "[%s\t\t*)"}.get(op)
        if rng is None:
            raise PqlCompilationException("unsupported operator %s" % op)
        return {"operator": "RANGE", "column": col, "values": [rng % v]}


def _flatten(op, kids):
    out = []
    for k in kids:
        if k.get("operator") == op and "children" in k:
            out.extend(k["children"])
        else:
            out.append(k)
    return {"operator": op, "children": out}


def compile_pql(text):
    """Compile a PQL query string into the query dict used by the executor (and the test oracle)."""
    return _Parser(_tokenize(text)).query()
