"""Resolves preprocessor conditionals on fixed macro values (a small unifdef).

    python tools/unifdef.py -DHL_X=0 -DHL_Y=1 file ...   (in place)

Every #if / #ifdef / #ifndef / #elif whose condition is decided by the given
macros is removed together with its dead branch; a condition that is only
partly decided keeps its directive with the decided operands dropped
(`defined(__HIP_DEVICE_COMPILE__) && HL_Y` -> `defined(__HIP_DEVICE_COMPILE__)`).
Development tool (round 6: measured-and-rejected variants pruned from the
kernel source, tools/patches/r06_pruned_variants.patch restores them).
"""
import re
import sys

TOK = re.compile(r"\s*(\|\||&&|==|!=|>=|<=|[()!<>]|defined\b|[A-Za-z_][A-Za-z0-9_]*|\d+)")


class Expr:
    """(value, text): value an int when decided, None when not; text the
    simplified expression."""

    def __init__(self, known, src):
        self.known, self.toks, self.i = known, TOK.findall(src), 0

    def peek(self):
        return self.toks[self.i].strip() if self.i < len(self.toks) else None

    def take(self):
        t = self.peek()
        self.i += 1
        return t

    def parse(self):
        v = self.orx()
        assert self.peek() is None, f"trailing tokens {self.toks[self.i:]}"
        return v

    def orx(self):
        a = self.andx()
        while self.peek() == "||":
            self.take()
            b = self.andx()
            if a[0] is not None and a[0]:
                a = (1, "1")
            elif b[0] is not None and b[0]:
                a = (1, "1")
            elif a[0] is not None:
                a = b
            elif b[0] is not None:
                pass
            else:
                a = (None, f"{a[1]} || {b[1]}")
        return a

    def andx(self):
        a = self.cmp()
        while self.peek() == "&&":
            self.take()
            b = self.cmp()
            if (a[0] is not None and not a[0]) or (b[0] is not None and not b[0]):
                a = (0, "0")
            elif a[0] is not None:
                a = b
            elif b[0] is not None:
                pass
            else:
                a = (None, f"{a[1]} && {b[1]}")
        return a

    def cmp(self):
        a = self.unary()
        if self.peek() in ("==", "!=", ">=", "<=", "<", ">"):
            op = self.take()
            b = self.unary()
            if a[0] is not None and b[0] is not None:
                return (int(eval(f"{a[0]} {op} {b[0]}")), None)
            return (None, f"{a[1]} {op} {b[1]}")
        return a

    def unary(self):
        if self.peek() == "!":
            self.take()
            v = self.unary()
            return (int(not v[0]), None) if v[0] is not None else (None, f"!{v[1]}")
        return self.primary()

    def primary(self):
        t = self.take()
        if t == "(":
            v = self.orx()
            assert self.take() == ")"
            return v if v[0] is not None or " " not in v[1] else (None, f"({v[1]})")
        if t == "defined":
            paren = self.peek() == "("
            if paren:
                self.take()
            name = self.take()
            if paren:
                assert self.take() == ")"
            return (1, None) if name in self.known else (None, f"defined({name})")
        if t.isdigit():
            return (int(t), t)
        if t in self.known:
            return (self.known[t], None)
        return (None, t)


def process(path, known):
    out, stack = [], []  # frame: [mode, taking, any_taken]; mode "res" (resolved) or "keep"
    live = lambda: all(f[1] for f in stack if f[0] == "res")  # noqa: E731
    for ln in open(path).read().split("\n"):
        m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", ln)
        if not m:
            if live():
                out.append(ln)
            continue
        d, rest = m.group(1), re.sub(r"//.*$|/\*.*?\*/", "", m.group(2)).strip()
        if d in ("if", "ifdef", "ifndef"):
            if not live():
                stack.append(["res", False, True])  # inside a dead branch: skip it whole
                continue
            src = rest if d == "if" else (f"defined({rest})" if d == "ifdef" else f"!defined({rest})")
            v, txt = Expr(known, src).parse()
            if v is None:
                stack.append(["keep", True, True])
                out.append(ln if d != "if" or txt == src else re.sub(r"(#\s*if\b).*", lambda mm: f"{mm.group(1)} {txt}", ln, count=1))
            else:
                stack.append(["res", bool(v), bool(v)])
        elif d == "elif":
            f = stack[-1]
            if f[0] == "keep":
                v, _ = Expr(known, rest).parse()
                assert v is None, f"{path}: #elif decided inside a kept conditional: {ln}"
                if live():
                    out.append(ln)
            else:
                if f[2]:
                    f[1] = False
                else:
                    v, _ = Expr(known, rest).parse()
                    assert v is not None, f"{path}: undecided #elif after a resolved #if: {ln}"
                    f[1] = f[2] = bool(v)
        elif d == "else":
            f = stack[-1]
            if f[0] == "keep":
                if live():
                    out.append(ln)
            else:
                f[1] = not f[2]
                f[2] = True
        else:  # endif
            f = stack.pop()
            if f[0] == "keep" and live():
                out.append(ln)
    assert not stack, f"{path}: unbalanced conditionals"
    open(path, "w").write("\n".join(out))


def main():
    known = {}
    files = []
    for a in sys.argv[1:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            known[k] = int(v or 1)
        else:
            files.append(a)
    for f in files:
        process(f, known)


if __name__ == "__main__":
    main()
