"""Generates the golden fixtures under tests/golden/ (committed; rerun to refresh).

    python tests/golden/make_golden.py

Two kinds of vectors:
  1. kat_*.json -- the reference's own known-answer tests, transcribed as data
     (inputs and expected outputs exactly as asserted in /root/reference/test/*,
     each entry citing its file:line).  No reference source is copied: only the
     asserted values.
  2. synth_*.json -- seeded workloads (emqx_amd.gen) whose expected per-topic
     match sets come from the oracle restatement (oracle/oracle.py) and are
     asserted here to equal brute-force emqx_topic:match/2 over every filter.
"""

from __future__ import annotations

import json
import os
import sys
from dataclasses import replace

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from emqx_amd import gen  # noqa: E402
from oracle import oracle as O  # noqa: E402


def b64(x: bytes) -> str:
    return x.decode("latin-1")


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


# ---------------------------------------------------------------- KATs

KAT_TOPIC = {
    "source": "test/emqx_topic_SUITE.erl",
    # [name, filter, expected]  emqx_topic:match/2
    "match": [
        # t_match1 :48-61
        ["a/b/c", "a/b/+", True], ["a/b/c", "a/#", True], ["abcd/ef/g", "#", True],
        ["abc/de/f", "abc/de/f", True], ["abc", "+", True], ["a/b/c", "a/b/c", True],
        ["a/b/c", "a/c/d", False], ["$share/x/y", "+", False], ["$share/x/y", "+/x/y", False],
        ["$share/x/y", "#", False], ["$share/x/y", "+/+/#", False], ["house/1/sensor/0", "house/+", False],
        ["house", "house/+", False],
        # t_match2 :63-80
        ["sport/tennis/player1", "sport/tennis/player1/#", True],
        ["sport/tennis/player1/ranking", "sport/tennis/player1/#", True],
        ["sport/tennis/player1/score/wimbledon", "sport/tennis/player1/#", True],
        ["sport", "sport/#", True], ["sport", "#", True], ["/sport/football/score/1", "#", True],
        ["Topic/C", "+/+", True], ["TopicA/B", "+/+", True], ["TopicA/C", "+/+", True],
        # t_match3 :82-88
        ["device/60019423a83c/fw", "device/60019423a83c/#", True],
        ["device/60019423a83c/$fw", "device/60019423a83c/#", True],
        ["device/60019423a83c/$fw/fw", "device/60019423a83c/$fw/#", True],
        ["device/60019423a83c/fw/checksum", "device/60019423a83c/#", True],
        ["device/60019423a83c/$fw/checksum", "device/60019423a83c/#", True],
        ["device/60019423a83c/dust/type", "device/60019423a83c/#", True],
        # t_sigle_level_match :90-99
        ["sport/tennis/player1", "sport/tennis/+", True],
        ["sport/tennis/player1/ranking", "sport/tennis/+", False],
        ["sport", "sport/+", False], ["sport/", "sport/+", True], ["/finance", "+/+", True],
        ["/finance", "/+", True], ["/finance", "+", False], ["/devices/$dev1", "/devices/+", True],
        ["/devices/$dev1/online", "/devices/+/online", True],
        # t_sys_match :101-105
        ["$SYS/broker/clients/testclient", "$SYS/#", True], ["$SYS/broker", "$SYS/+", True],
        ["$SYS/broker", "+/+", False], ["$SYS/broker", "#", False],
        # 't_#_match' :107-112
        ["a/b/c", "#", True], ["a/b/c", "+/#", True], ["$SYS/brokers", "#", False],
        ["a/b/$c", "a/b/#", True], ["a/b/$c", "a/#", True],
        # t_match_perf :114-119
        ["a/b/ccc", "a/#", True],
        ["/abkc/19383/192939/akakdkkdkak/xxxyyuya/akakak", "/abkc/19383/+/akakdkkdkak/#", True],
        # test/emqx_client_SUITE.erl:166-186 (overlapping) and :234-247 ($ topics)
        ["TopicA/C", "TopicA/#", True], ["TopicA/C", "TopicA/+", True], ["$TopicA/B", "+/+", False],
    ],
    # t_wildcard :42-46
    "wildcard": [["a/b/#", True], ["a/+/#", True], ["", False], ["a/b/c", False]],
    # t_words :160-166 (atoms written as "'+'" etc.)
    "words": [["/a/+/#", ["''", "a", "'+'", "'#'"]],
              ["/abkc/19383/+/akakdkkdkak/#", ["''", "abkc", "19383", "'+'", "akakdkkdkak", "'#'"]]],
    # t_tokens :156-158, t_levels :152-154
    "tokens": [["a/b/+/#", ["a", "b", "+", "#"]]],
    "levels": [["a/+/#", 3], ["a/b/c/d", 4]],
    # t_validate :121-137, t_sigle_level_validate :139-143 -> [kind, topic, "ok" | error reason]
    "validate": [
        ["filter", "a/+/#", "ok"], ["filter", "a/b/c/d", "ok"], ["name", "abc/de/f", "ok"],
        ["filter", "abc/+/f", "ok"], ["filter", "abc/#", "ok"], ["filter", "x", "ok"], ["name", "x//y", "ok"],
        ["filter", "sport/tennis/#", "ok"], ["name", "", "empty_topic"], ["name", "abc/#", "topic_name_error"],
        ["name", "LONG", "topic_too_long"], ["filter", "abc/#/1", "topic_invalid_#"],
        ["filter", "abc/#xzy/+", "topic_invalid_char"], ["filter", "abc/xzy/+9827", "topic_invalid_char"],
        ["filter", "sport/tennis#", "topic_invalid_char"], ["filter", "sport/tennis/#/ranking", "topic_invalid_#"],
        ["filter", "+", "ok"], ["filter", "+/tennis/#", "ok"], ["filter", "sport/+/player1", "ok"],
        ["filter", "sport+", "topic_invalid_char"],
    ],
    # t_join :168-175 (words given as topics to be tokenised where the suite does so)
    "join": [[[], ""], [["x"], "x"], [["'#'"], "#"], [["'+'", "''", "'#'"], "+//#"],
             [["x", "y", "z", "'+'"], "x/y/z/+"]],
    "join_words": [["/ab/cd/ef/", "/ab/cd/ef/"], ["ab/+/#", "ab/+/#"]],
    # t_prepend :145-150
    "prepend": [[None, "ab", "ab"], ["", "a/b", "a/b"], ["x/", "a/b", "x/a/b"], ["x/y", "a/b", "x/y/a/b"],
                ["'+'", "a/b", "+/a/b"]],
    # t_feed_var :184-191
    "feed_var": [["$c", "clientId", "$queue/client/$c", "$queue/client/clientId"],
                 ["%u", "test", "username/%u/client/x", "username/test/client/x"],
                 ["%c", "clientId", "username/test/client/%c", "username/test/client/clientId"]],
    # t_parse :196-216 -> [input, options, expected filter | error, expected share]
    "parse": [["$queue/t", {"share": "g"}, "error", None], ["$share/g/t", {"share": "g"}, "error", None],
              ["$share/t", {}, "error", None], ["$share/+/t", {}, "error", None],
              ["a/b/+/#", {}, "a/b/+/#", None], ["$queue/topic", {}, "topic", "$queue"],
              ["$share/group/topic", {}, "topic", "group"], ["$local/topic", {}, "$local/topic", None],
              ["$local/$queue/topic", {}, "$local/$queue/topic", None],
              ["$local/$share/group/a/b/c", {}, "$local/$share/group/a/b/c", None],
              ["$fastlane/topic", {}, "$fastlane/topic", None]],
}

# test/emqx_trie_SUITE.erl -- sequences of ops; "match" results are in the
# reference's own (DFS) order, "sorted" is the build's contract.
KAT_TRIE = {
    "source": "test/emqx_trie_SUITE.erl",
    "cases": [
        {"name": "t_insert", "line": "49-63",
         "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"],
                 ["insert", "sensor"], ["insert", "sensor"]],
         "lookup": [["sensor", [3, "sensor"]]]},
        {"name": "t_match", "line": "65-73",
         "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"]],
         "match": [["sensor/1", ["sensor/+/#", "sensor/#"]]]},
        {"name": "t_match2", "line": "75-84",
         "ops": [["insert", "#"], ["insert", "+/#"], ["insert", "+/+/#"]],
         "match": [["a/b/c", ["+/+/#", "+/#", "#"]], ["$SYS/broker/zenmq", []]]},
        {"name": "t_match3", "line": "86-92",
         "ops": [["insert", t] for t in ["d/#", "a/b/c", "a/b/+", "a/#", "#", "$SYS/#"]],
         "match_len": [["a/b/c", 4]], "match": [["$SYS/a/b/c", ["$SYS/#"]]]},
        {"name": "t_empty", "line": "94-99",
         "ops": [["empty", True], ["insert", "topic/x/#"], ["empty", False], ["delete", "topic/x/#"],
                 ["empty", True]]},
        {"name": "t_delete", "line": "101-115",
         "ops": [["insert", "sensor/1/#"], ["insert", "sensor/1/metric/2"], ["insert", "sensor/1/metric/3"],
                 ["delete", "sensor/1/metric/2"], ["delete", "sensor/1/metric"], ["delete", "sensor/1/metric"]],
         "lookup": [["sensor/1", [2, None]]]},
        {"name": "t_delete2", "line": "117-128",
         "ops": [["insert", "sensor"], ["insert", "sensor/1/metric/2"], ["insert", "sensor/+/metric/3"],
                 ["delete", "sensor"], ["delete", "sensor/1/metric/2"], ["delete", "sensor/+/metric/3"],
                 ["delete", "sensor/+/metric/3"]],
         "lookup": [["sensor", None], ["sensor/1", None]]},
        {"name": "t_delete3", "line": "130-142",
         "ops": [["insert", "sensor/+"], ["insert", "sensor/+/metric/2"], ["insert", "sensor/+/metric/3"],
                 ["delete", "sensor/+/metric/2"], ["delete", "sensor/+/metric/3"], ["delete", "sensor"],
                 ["delete", "sensor/+"], ["delete", "sensor/+/unknown"]],
         "lookup": [["sensor", None], ["sensor/+", None]]},
    ],
    # t_triples :144-148
    "triples": [["a/b/c", [["root", "a", "a"], ["a", "b", "a/b"], ["a/b", "c", "a/b/c"]]]],
}

KAT_BROKER = {
    "source": "test/emqx_broker_SUITE.erl, test/emqx_client_SUITE.erl",
    "note": "ops: sub/unsub/down change the subscriber bag; pub lists the deliveries "
            "[filter, subscriber] of one publish (filters in binary order); "
            "subscribers/topics are the table reads the tests assert",
    "cases": [
        {"name": "t_subscribers", "line": "emqx_broker_SUITE.erl:92-95",
         "ops": [["sub", "topic", "self"], ["subscribers", "topic", ["self"]], ["unsub", "topic", "self"],
                 ["subscribers", "topic", []]]},
        {"name": "t_sub_pub", "line": "emqx_broker_SUITE.erl:106-118",
         "ops": [["sub", "topic", "self"], ["pub", "topic", [["topic", "self"]]]]},
        {"name": "t_nosub_pub", "line": "emqx_broker_SUITE.erl:120-123",
         "ops": [["pub", "topic", []]]},
        {"name": "t_shard", "line": "emqx_broker_SUITE.erl:177-192",
         "ops": [["sub", "topic", "clientid"], ["pub", "topic", [["topic", "clientid"]]]]},
        {"name": "t_topics", "line": "emqx_broker_SUITE.erl:76-90",
         "ops": [["sub", "topic", "clientId"], ["sub", "topic/1", "clientId"], ["sub", "topic/2", "clientId"],
                 ["topics", ["topic", "topic/1", "topic/2"]],
                 ["unsub", "topic", "clientId"], ["unsub", "topic/1", "clientId"], ["unsub", "topic/2", "clientId"],
                 ["topics", []]]},
        {"name": "t_overlapping_subscriptions", "line": "emqx_client_SUITE.erl:166-186",
         "note": "this broker publishes one message per matching subscription (Num == 2)",
         "ops": [["sub", "TopicA/#", "C"], ["sub", "TopicA/+", "C"],
                 ["pub", "TopicA/C", [["TopicA/#", "C"], ["TopicA/+", "C"]]]]},
        {"name": "t_dollar_topics", "line": "emqx_client_SUITE.erl:234-247",
         "ops": [["sub", "+/+", "C"], ["pub", "$TopicA/B", []]]},
    ],
}


KAT_ROUTER = {
    "source": "test/emqx_router_SUITE.erl",
    "cases": [
        {"name": "t_add_delete", "line": "66-73",
         "add": ["a/b/c", "a/b/c", "a/+/b"], "topics": ["a/+/b", "a/b/c"],
         "delete": ["a/b/c", "a/+/b"], "topics_after": []},
        {"name": "t_match_routes", "line": "85-99",
         "add": ["a/b/c", "a/+/c", "a/b/#", "#"], "match": ["a/b/c", ["#", "a/+/c", "a/b/#", "a/b/c"]],
         "delete": ["a/b/c", "a/+/c", "a/b/#", "#"], "match_after": ["a/b/c", []]},
        {"name": "t_has_routes", "line": "106-109", "add": ["devices/+/messages"],
         "has": ["devices/+/messages", True]},
    ],
}

KAT_BATCH = {
    "source": "test/emqx_batch_SUITE.erl",
    "note": "steps run in order against init(opts); 'commits' = the lists commit_fun received, in order",
    "cases": [
        {"name": "t_batch_full_commit", "line": "26-37", "opts": {"batch_size": 3, "linger_ms": 2000},
         "steps": [{"push": "a"}, {"push": "b"}, {"push": "c"},
                   {"size": 3, "items": ["a", "b", "c"]},
                   {"push": "a"},          # 4th push onto 3 queued items: commit at batch_size + 1
                   {"size": 0, "items": []}],
         "commits": [["a", "b", "c", "a"]]},
        {"name": "t_batch_linger_commit", "line": "39-56", "opts": {"batch_size": 3, "linger_ms": 500},
         "steps": [{"push": "a"}, {"push": "b"}, {"push": "c"},
                   {"size": 3, "items": ["a", "b", "c"]},
                   {"await_linger_within_ms": 1000},   # batch_linger_expired arrives
                   {"commit": True},
                   {"size": 0, "items": []}],
         "commits": [["a", "b", "c"]]},
        # src/emqx_batch.erl:64-66 (no suite case): batch_size = 0 never commits on push
        {"name": "src_unlimited", "line": "src/emqx_batch.erl:64-66", "opts": {"batch_size": 0, "linger_ms": 60000},
         "steps": [{"push": "a"}, {"push": "b"}, {"push": "c"}, {"push": "d"},
                   {"size": 4, "items": ["a", "b", "c", "d"]}],
         "commits": []},
    ],
}

# Hand-written adversarial filters/topics: byte classes around '#' (0x23) and
# '+' (0x2B), empty levels, '$' rules, literal '#'/'+' topic words, deep topics,
# irregular '+x' words, shared-prefix filters.
ADV_FILTERS = [
    "#", "+", "+/#", "+/+", "/+", "/#", "+//#", "//#", "a", "a/", "a//", "a/#", "a/+", "a/+/#", "a//#",
    "a/b", "a/b/#", "a/b/+", "a/+/c", "a/!x", "a/!x/#", "a/%x", "a/%x/#", "a/$x", "a/$x/#", "a/ x", "a/ x/+",
    "a/#x", "a/#/b", "a/+/+", "a//b", "a//+", "$SYS/#", "$SYS/+", "$SYS/a/+", "$SYS", "+/b/#", "a/b/c/d/e/f/g/h/i/j/k/l",
    "a/+/c/+/e/+/g/+/i/+/k/#", "x/y", "x/y/", "x/y//", "x/y/#", "x/+/", "x/+/+", "/", "//", "///", "+/", "/+/",
    "#/#", "a/#/#", "+/+/+/+/+/+/+/+/+/+/+/+", "+/+/+/+/+/+/+/+/+/+/+", "u/v/w/x/y/z/#", "!", "%", "~", "a/~",
    "a/b/c", "a/b/c/#", "a/b/c/+", "a/+x", "a/+x/#", "a/x+", "e", "e/", "e/#", "e/+", "é/#", "é/ü/+",
]
ADV_TOPICS = [
    "a", "a/", "a//", "a/b", "a/b/c", "a/b/c/d", "a/!x", "a/%x", "a/$x", "a/ x", "a/#x", "a/x", "a//b",
    "/", "//", "///", "/a", "//a", "$SYS", "$SYS/a", "$SYS/a/b", "$x/y", "x/y", "x/y/", "x/y//", "x/z/",
    "a/b/c/d/e/f/g/h/i/j/k/l", "a/b/c/d/e/f/g/h/i/j/k", "a/z/c/z/e/z/g/z/i/z/k/z/m", "a/#", "a/+", "a/#/b",
    "+", "#", "+/+", "a/+/c", "a/b/#", "u/v/w/x/y/z", "u/v/w/x/y/z/1/2/3/4/5/6/7/8/9/0/1/2/3/4/5/6",
    "!", "%", "~", "a/~", "e", "e/", "é", "é/ü/ö", "a/+x", "a/+x/y", "a/x+", "q/r/s/t/u/v/w/x/y/z/a/b/c/d/e/f/g/h/i/j/k",
]


def synth(name, p: gen.Params, n_topics: int, tseed: int, extra_filters=(), extra_topics=()):
    F = gen.py_gen_filters(p) + [f.encode() for f in extra_filters]
    F = list(dict.fromkeys(F))
    T = gen.py_gen_topics(p, F, tseed, n_topics) + [t.encode() for t in extra_topics]
    tr = O.Trie()
    for f in F:
        tr.insert(f)
    rows = []
    for t in T:
        got = sorted(set(tr.match(t)))   # the reference lists duplicates for wildcard names
        if not O.wildcard(t):
            # valid publish names: two independent formulations must agree.  (For
            # names holding '+'/'#' words the reference's match/2 and trie walk
            # differ -- e.g. "a/#/b" vs "a/#" -- and the hot path is the trie.)
            exp = O.brute(t, F)
            assert got == exp, (t, got, exp)
        idx = {f: i for i, f in enumerate(F)}
        rows.append([idx[f] for f in got])
    dump(name, {"params": {k: getattr(p, k) for k in p.__dataclass_fields__}, "tseed": tseed,
                "filters": [b64(f) for f in F], "topics": [b64(t) for t in T], "expected": rows,
                "note": "expected[i] = indices into filters, sorted by filter bytes (Erlang binary order); "
                        "generated by oracle/oracle.py, asserted equal to brute-force emqx_topic:match/2"})


def main():
    dump("kat_topic.json", KAT_TOPIC)
    dump("kat_trie.json", KAT_TRIE)
    dump("kat_router.json", KAT_ROUTER)
    dump("kat_broker.json", KAT_BROKER)
    dump("kat_batch.json", KAT_BATCH)
    synth("synth_c1_small.json", replace(gen.C1, n_filters=800), 600, 11)
    synth("synth_c2_small.json", replace(gen.C2, n_filters=1500, vocab=48), 600, 22)
    synth("synth_adversarial.json", replace(gen.C1, n_filters=150, vocab=6, p_empty=0.2, p_dollar=0.1), 300, 33,
          ADV_FILTERS, ADV_TOPICS)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
