"""emqx_shared_sub mirror: the routes of shared subscriptions.

A shared subscription `$share/Group/Topic` is routed as `#route{topic = Topic,
dest = {Group, node()}}`: the group's first member on a node adds that route and
its last member (unsubscribe or process down) deletes it
(src/emqx_shared_sub.erl:297-315, 358-367).  On the device the route aggregates
to the Group (emqx_broker:aggre/1, src/emqx_broker.erl:250-261), so
`emqx_router.aggre_batch` returns `(To, Group)` pairs for it.

Which member receives a message (the random / round_robin / sticky / hash
strategies, :115-129, 229-275) is decided per delivery by the group's dispatcher
process and is not part of the matching path.
"""

from __future__ import annotations

from . import emqx_router as R

_members = {}   # (group, topic) -> [subpid] (?SHARED_SUBS bag, insertion order)
_of_pid = {}    # subpid -> [(group, topic)] (the mnesia ?TAB records of the pid)


def clear():
    _members.clear()
    _of_pid.clear()


def subscribe(group, topic: bytes, subpid, node=R.NODE):
    """handle_call({subscribe, Group, Topic, SubPid}) (:297-305)."""
    topic = bytes(topic)
    key = (group, topic)
    ms = _members.get(key)
    if ms is None:                                    # not ets:member(?SHARED_SUBS, {Group, Topic})
        R.do_add_route(topic, (group, node))
        ms = _members[key] = []
    if subpid not in ms:                              # a bag stores an identical object once
        ms.append(subpid)
        _of_pid.setdefault(subpid, []).append(key)
    return "ok"


def unsubscribe(group, topic: bytes, subpid, node=R.NODE):
    """handle_call({unsubscribe, Group, Topic, SubPid}) (:307-315)."""
    key = (group, bytes(topic))
    ms = _members.get(key)
    if ms and subpid in ms:
        ms.remove(subpid)
        ks = _of_pid[subpid]
        ks.remove(key)
        if not ks:
            del _of_pid[subpid]
    if key in _members and not _members[key]:
        del _members[key]
        R.do_delete_route(key[1], (group, node))
    return "ok"


def member_down(subpid, node=R.NODE) -> int:
    """cleanup_down/1 (:358-367) on the subscriber's 'DOWN'."""
    keys = list(_of_pid.get(subpid, []))
    for g, t in keys:
        unsubscribe(g, t, subpid, node)
    return len(keys)


def subscribers(group, topic: bytes):
    """subscribers/2: the group's members for the topic."""
    return list(_members.get((group, bytes(topic)), []))
