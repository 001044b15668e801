"""Batch topic -> rule matching for the rule engine and authz.

The reference evaluates these by linear scans of the emqx_topic:match/2
predicate per message:
  * rule engine: get_rules_for_topic/1 keeps every rule with a FROM filter
    that matches (apps/emqx_rule_engine/src/emqx_rule_engine.erl:162-165 ->
    emqx_plugin_libs_rule:can_topic_match_oneof/2,
    apps/emqx_plugin_libs/src/emqx_plugin_libs_rule.erl:265-268);
  * authz: emqx_authz_rule:matches/4 returns the first rule (in order) whose
    action, who and topic filters match (apps/emqx_authz/src/emqx_authz_rule.erl:
    110-125, 167-180); a filter is a pattern or {eq, Topic} (literal equality,
    :82-85).

Here the distinct filters of all rules form one GPU index; a batch of publish
topics is matched once (emqx_gm_match with match_routes semantics, which for a
topic NAME is exactly {F : emqx_topic:match(Name, F)}), and the per-filter rule
lists are gathered on the device by emqx_gm_fanout (filter -> rule indices play
the role of the subscriber lists).  Only topic names are accepted: for a name
with '+'/'#' words (an authz subscribe check) emqx_topic:match/2 compares
wildcards word by word, which is not the publish semantics served here.
An {eq, F} filter equals pattern F for names when F has no wildcard, and never
matches a name when it has one.  Client placeholders (%u, %c) must be resolved
by the caller.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import topic as T
from .engine import Context, Index

Filter = Union[bytes, str, Tuple[str, Union[bytes, str]]]


def _b(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


class TopicRuleIndex:
    """rules[i] = the topic filters of rule i (bytes/str patterns or ("eq", topic))."""

    def __init__(self, ctx: Context, rules: Sequence[Sequence[Filter]]):
        self.ctx = ctx
        self.n_rules = len(rules)
        owners = {}
        for r, fs in enumerate(rules):
            for f in fs:
                if isinstance(f, tuple):
                    kind, lit = f
                    if kind != "eq":
                        raise ValueError(f"unknown filter form {kind!r}")
                    lit = _b(lit)
                    if T.wildcard(lit):
                        continue  # {eq, 'a/+'} only equals the name 'a/+', never a topic name
                    f = lit
                else:
                    f = _b(f)
                owners.setdefault(f, set()).add(r)
        self.filters = sorted(owners)
        self.index: Index = ctx.build_index(self.filters, subs=[sorted(owners[f]) for f in self.filters])

    def rules_for_topics(self, topics: Sequence) -> List[List[int]]:
        """Per topic, the ascending indices of the rules with a matching filter
        (get_rules_for_topic/1 over a batch)."""
        names = [_b(t) for t in topics]
        for t in names:
            if T.wildcard(t):
                raise ValueError(f"topic names only (got filter {t!r})")
        (ro, ids), (fro, rids) = self.ctx.match_fanout(self.index, names, exact=True)
        out = []
        for k in range(len(names)):
            out.append(np.unique(rids[fro[k]:fro[k + 1]]).astype(np.int64).tolist())
        return out

    def first_match(self, topics: Sequence, eligible: Optional[Sequence[bool]] = None) -> List[int]:
        """Per topic, the first rule (in rule order) whose topic filters match and
        that is eligible (its action and who already matched: matches/4), or -1."""
        rows = self.rules_for_topics(topics)
        out = []
        for row in rows:
            hit = -1
            for r in row:  # ascending = rule order
                if eligible is None or eligible[r]:
                    hit = r
                    break
            out.append(hit)
        return out

    def release(self):
        self.index.release()
