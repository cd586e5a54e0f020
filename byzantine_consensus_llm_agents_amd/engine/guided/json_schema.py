"""JSON Schema -> byte-level regular AST (the language guided decoding enforces).

Covers what the BCG agents use and the common rest:
objects (properties emitted in schema order, required/optional,
``additionalProperties: false``), strings (full JSON escapes, UTF-8
validated, optional ``enum``/``maxLength``), integers with exact
``minimum``/``maximum`` ranges, numbers, booleans, null, arrays, ``anyOf`` /
``oneOf`` / ``enum`` / ``const``.

Whitespace between structural tokens is limited to ``max_ws`` bytes of
``[ \\t\\n\\r]`` so the language stays finite-state and an untrained model
cannot loop forever inside whitespace.
"""

import json
from itertools import combinations
from typing import Any, Dict, List

from .regex_dfa import (Cls, Lit, Node, Rep, Star, alt, byte_mask, chars_mask, compile_dfa, lit, seq)

DIGIT = Cls(byte_mask((0x30, 0x39)))
NONZERO = Cls(byte_mask((0x31, 0x39)))
HEX = Cls(byte_mask((0x30, 0x39), (0x41, 0x46), (0x61, 0x66)))
CONT = Cls(byte_mask((0x80, 0xBF)))


def _string_char_parts() -> List[Node]:
    """The alternatives of one JSON string character other than plain ASCII: an escape, and
    2- / 3- / 4-byte UTF-8 sequences."""
    escape = seq(lit("\\"), alt(Cls(chars_mask(b'"\\/bfnrt')), seq(lit("u"), HEX, HEX, HEX, HEX)))
    two = seq(Cls(byte_mask((0xC2, 0xDF))), CONT)
    three = alt(seq(lit(b"\xe0"), Cls(byte_mask((0xA0, 0xBF))), CONT),
                seq(Cls(byte_mask((0xE1, 0xEC))), CONT, CONT),
                seq(lit(b"\xed"), Cls(byte_mask((0x80, 0x9F))), CONT),
                seq(Cls(byte_mask((0xEE, 0xEF))), CONT, CONT))
    four = alt(seq(lit(b"\xf0"), Cls(byte_mask((0x90, 0xBF))), CONT, CONT),
               seq(Cls(byte_mask((0xF1, 0xF3))), CONT, CONT, CONT),
               seq(lit(b"\xf4"), Cls(byte_mask((0x80, 0x8F))), CONT, CONT))
    return [escape, two, three, four]


_STRING_CHAR_NON_ASCII = _string_char_parts()
STRING_CHAR = alt(Cls(byte_mask((0x20, 0x7F)) & ~chars_mask(b'"\\')), *_STRING_CHAR_NON_ASCII)
# a character Python's str.strip() never removes: printable ASCII other than space (and the
# two that need escaping); escapes and non-ASCII characters do not count as visible
VISIBLE_CHAR = Cls(byte_mask((0x21, 0x7E)) & ~chars_mask(b'"\\'))

# printable ASCII without the two characters that need escaping: the free text of the benchmark's
# ASCII grammar (no escapes, no multi-byte UTF-8)
ASCII_TEXT_CHAR = Cls(byte_mask((0x20, 0x7E)) & ~chars_mask(b'"\\'))

# JSON-schema extension keywords of the benchmark's validity-aware grammar: a string carries at
# least this many visible characters (VISIBLE_CHAR), anywhere in it; and (ASCII_TEXT) its
# characters are printable ASCII only
MIN_VISIBLE = "x-min-visible"
ASCII_TEXT = "x-ascii-text"


def validity_aware(schema: Dict, min_visible: int = 10, ascii_text: bool = False) -> Dict:
    """The benchmark grammar for untrained weights (engine option ``validity_aware_json``):
    every object property is emitted (optional ones made required) and every free-text string
    (no enum / const) carries >= `min_visible` visible characters -- the simulator's own validity
    rules for a decision (strategy >= 3, reasoning >= 10 stripped characters, reference
    main.py:232-247) then hold for every output, as they do for a trained model's; a random
    model under the plain grammar closes strings early or skips optional fields, and those
    outputs go down the retry ladder.

    `ascii_text`: free text is printable ASCII (no escapes, no multi-byte UTF-8), as an
    English-speaking trained model writes it.  A random model otherwise emits escapes and
    multi-byte characters that re-tokenise at several tokens per character once the game
    quotes them in later prompts (reasoning [:200], strategies 5 x 400 chars), and late-game
    prompts run into the context limit -- far outside the reference's bounded prompt sizes
    (~0.6-2.5k tokens).  Idempotent (TP followers re-apply it to the key)."""
    if not isinstance(schema, dict):
        return schema
    out = dict(schema)
    for key in ("anyOf", "oneOf"):
        if key in out:
            out[key] = [validity_aware(s, min_visible, ascii_text) for s in out[key]]
    if out.get("type") == "object" and "properties" in out:
        out["properties"] = {k: validity_aware(v, min_visible, ascii_text) for k, v in out["properties"].items()}
        out["required"] = list(out["properties"])
    if out.get("type") == "string" and "enum" not in out and "const" not in out:
        out[MIN_VISIBLE] = max(int(out.get(MIN_VISIBLE, 0)), min_visible)
        if ascii_text:
            out[ASCII_TEXT] = True
    return out


def _same_len_range(a: str, b: str) -> Node:
    """Decimal strings of equal length between a and b (inclusive)."""
    if len(a) == 1:
        return Cls(byte_mask((ord(a), ord(b))))
    if a[0] == b[0]:
        return seq(lit(a[0]), _same_len_range(a[1:], b[1:]))
    n = len(a) - 1
    parts = [seq(lit(a[0]), _same_len_range(a[1:], "9" * n)),
             seq(lit(b[0]), _same_len_range("0" * n, b[1:]))]
    if ord(b[0]) - ord(a[0]) > 1:
        parts.insert(1, seq(Cls(byte_mask((ord(a[0]) + 1, ord(b[0]) - 1))), *([DIGIT] * n)))
    return alt(*parts)


def _nonneg_range(lo: int, hi: int) -> Node:
    opts = []
    for width in range(len(str(lo)), len(str(hi)) + 1):
        start = max(lo, 10 ** (width - 1) if width > 1 else 0)
        stop = min(hi, 10 ** width - 1)
        if start <= stop:
            opts.append(_same_len_range(str(start), str(stop)))
    return alt(*opts)


def integer_node(minimum=None, maximum=None) -> Node:
    if minimum is None or maximum is None:
        unsigned = alt(lit("0"), seq(NONZERO, Star(DIGIT)))
        if minimum is not None and minimum >= 0:
            return unsigned
        return seq(Rep(lit("-"), 0, 1), unsigned)
    lo, hi = int(minimum), int(maximum)
    if lo > hi:
        raise ValueError(f"empty integer range [{lo}, {hi}]")
    opts = []
    if lo < 0:
        neg_hi, neg_lo = -lo, max(1, -min(hi, -1))
        opts.append(seq(lit("-"), _nonneg_range(neg_lo, neg_hi)))
    if hi >= 0:
        opts.append(_nonneg_range(max(lo, 0), hi))
    return alt(*opts)


NUMBER = seq(Rep(lit("-"), 0, 1), alt(lit("0"), seq(NONZERO, Star(DIGIT))),
             Rep(seq(lit("."), DIGIT, Star(DIGIT)), 0, 1),
             Rep(seq(Cls(chars_mask(b"eE")), Rep(Cls(chars_mask(b"+-")), 0, 1), DIGIT, Star(DIGIT)), 0, 1))


class SchemaCompiler:
    def __init__(self, max_ws: int = 4):
        self.max_ws = max_ws
        self.ws = Rep(Cls(chars_mask(b" \t\n\r")), 0, max_ws) if max_ws > 0 else lit("")

    def literal_value(self, value: Any) -> Node:
        return lit(json.dumps(value, ensure_ascii=False))

    def node(self, schema: Dict) -> Node:
        if schema is True or schema == {}:
            return self.any_value(depth=2)
        if "const" in schema:
            return self.literal_value(schema["const"])
        if "enum" in schema:
            return alt(*[self.literal_value(v) for v in schema["enum"]])
        for key in ("anyOf", "oneOf"):
            if key in schema:
                return alt(*[self.node(s) for s in schema[key]])
        kind = schema.get("type")
        if isinstance(kind, list):
            return alt(*[self.node({**schema, "type": k}) for k in kind])
        if kind == "object":
            return self.object_node(schema)
        if kind == "string" and schema.get(MIN_VISIBLE):
            # (invisible chars* visible){k} then any chars: >= k visible characters
            k = int(schema[MIN_VISIBLE])
            if schema.get(ASCII_TEXT):
                invisible, char = lit(" "), ASCII_TEXT_CHAR
            else:
                invisible, char = alt(Cls(chars_mask(b" \x7f")), *_STRING_CHAR_NON_ASCII), STRING_CHAR
            body = seq(Rep(seq(Star(invisible), VISIBLE_CHAR), k, k), Star(char))
            return seq(lit('"'), body, lit('"'))
        if kind == "string" and schema.get(ASCII_TEXT) and "enum" not in schema:
            return seq(lit('"'), Star(ASCII_TEXT_CHAR), lit('"'))
        if kind == "string":
            n = schema.get("maxLength")
            body = Rep(STRING_CHAR, int(schema.get("minLength", 0)), int(n)) if n is not None else (
                Rep(STRING_CHAR, int(schema.get("minLength", 0)), -1))
            return seq(lit('"'), body, lit('"'))
        if kind == "integer":
            return integer_node(schema.get("minimum"), schema.get("maximum"))
        if kind == "number":
            return NUMBER
        if kind == "boolean":
            return alt(lit("true"), lit("false"))
        if kind == "null":
            return lit("null")
        if kind == "array":
            item = self.node(schema.get("items", {}))
            ws = self.ws
            more = Star(seq(ws, lit(","), ws, item))
            return seq(lit("["), ws, Rep(seq(item, more), 0, 1), ws, lit("]"))
        raise ValueError(f"unsupported schema: {schema}")

    def any_value(self, depth: int) -> Node:
        scalar = alt(seq(lit('"'), Star(STRING_CHAR), lit('"')), NUMBER, lit("true"), lit("false"), lit("null"))
        return scalar  # free-form objects are not needed by the BCG schemas

    def object_node(self, schema: Dict) -> Node:
        props = schema.get("properties", {})
        required = set(schema.get("required", []))
        names = list(props)
        ws = self.ws
        members = {n: seq(lit(json.dumps(n)), ws, lit(":"), ws, self.node(props[n])) for n in names}
        optional = [n for n in names if n not in required]
        variants: List[Node] = []
        # every subsequence that keeps all required properties, in schema order
        for k in range(len(optional) + 1):
            for dropped in combinations(optional, k):
                keep = [n for n in names if n not in dropped]
                if not keep:
                    variants.append(lit(""))
                    continue
                body = [members[keep[0]]]
                for n in keep[1:]:
                    body += [ws, lit(","), ws, members[n]]
                variants.append(seq(*body))
        return seq(lit("{"), ws, alt(*variants), ws, lit("}"))


def schema_to_dfa(schema: Dict, max_ws: int = 4):
    return compile_dfa(SchemaCompiler(max_ws).node(schema))
