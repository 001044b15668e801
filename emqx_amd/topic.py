"""Host mirror of emqx_topic (apps/emqx/src/emqx_topic.erl) used by the API layer.

These are per-topic utilities (validation, splitting, the match/2 predicate
for single pairs); the batch hot path is the GPU trie walk in engine.py.
Atoms '' / '+' / '#' are represented by the Python strings "", "+", "#";
other words are bytes.
"""

from __future__ import annotations

from typing import List, Sequence, Union

MAX_TOPIC_LEN = 65535  # emqx_topic.erl:45

Word = Union[bytes, str]


def _b(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


def tokens(topic) -> List[bytes]:
    """tokens/1 (:150-154): binary:split(T, <<"/">>, [global])."""
    return _b(topic).split(b"/")


def word(w: bytes) -> Word:
    """word/1 (:161-164)."""
    if w == b"":
        return ""
    if w == b"+":
        return "+"
    if w == b"#":
        return "#"
    return w


def words(topic) -> List[Word]:
    """words/1 (:157-159)."""
    return [word(w) for w in tokens(topic)]


def wildcard(topic) -> bool:
    """wildcard/1 (:52-62)."""
    ws = words(topic) if isinstance(topic, (bytes, bytearray, str)) else topic
    return any(w in ("+", "#") for w in ws)


def _bin(w: Word) -> bytes:
    return b"" if w == "" else b"+" if w == "+" else b"#" if w == "#" else _b(w)


def join(ws: Sequence[Word]) -> bytes:
    """join/1 (:183-195)."""
    return b"/".join(_bin(w) for w in ws)


def match(name, filt) -> bool:
    """match/2 (:65-87), including the '$' rule on the first byte."""
    n, f = _b(name), _b(filt)
    if n[:1] == b"$" and f[:1] in (b"+", b"#"):
        return False
    nw, fw = words(n), words(f)
    i = j = 0
    while True:
        if i == len(nw) and j == len(fw):               # match([], [])
            return True
        if i < len(nw) and j < len(fw) and (nw[i] == fw[j] or fw[j] == "+"):
            i += 1                                      # match([H|T1], [H|T2]) / ['+'|T2]
            j += 1
            continue
        return j + 1 == len(fw) and fw[j] == "#"        # match(_, ['#'])


class TopicError(ValueError):
    pass


def validate(topic, kind: str = "filter") -> bool:
    """validate/2 (:96-127): raises TopicError(reason) like error(Reason)."""
    t = _b(topic)
    if t == b"":
        raise TopicError("empty_topic")
    if len(t) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    ws = words(t)
    for k, w in enumerate(ws):
        if w == "#":
            if k != len(ws) - 1:
                raise TopicError("topic_invalid_#")
        elif isinstance(w, bytes) and (b"#" in w or b"+" in w or b"\0" in w):
            raise TopicError("topic_invalid_char")
    if kind == "name" and wildcard(ws):
        raise TopicError("topic_name_error")
    return True


def levels(topic) -> int:
    return len(tokens(topic))


def parse(topic_filter, options=None):
    """parse/2 (:197-220): strips $share/<group>/ and $queue/."""
    opts = dict(options or {})
    t = _b(topic_filter)
    if t.startswith(b"$queue/"):
        if "share" in opts:
            raise TopicError(("invalid_topic_filter", t))
        opts["share"] = b"$queue"
        return parse(t[len(b"$queue/"):], opts)
    if t.startswith(b"$share/"):
        if "share" in opts:
            raise TopicError(("invalid_topic_filter", t))
        rest = t[len(b"$share/"):]
        if b"/" not in rest:
            raise TopicError(("invalid_topic_filter", t))
        group, filt = rest.split(b"/", 1)
        if b"+" in group or b"#" in group:
            raise TopicError(("invalid_topic_filter", t))
        opts["share"] = group
        return parse(filt, opts)
    return t, opts
