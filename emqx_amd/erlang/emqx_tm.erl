%% emqx_tm -- Erlang face of the MI355X topic-matching engine (NIF: emqx_tm_nif.c).
%%
%% Drop-in for the read side of emqx_trie (src/emqx_trie.erl) used by
%% emqx_router:match_routes/1 (src/emqx_router.erl:127-141), plus the trie
%% mutations the router applies after its mnesia transaction commits.
%% See INTEGRATION.md for the two-line change in emqx_router.
-module(emqx_tm).

-export([ new/1
        , insert/2
        , delete/2
        , lookup/2
        , empty/1
        , match/2
        , match_async/3
        , match_batch/2
        , topic_match/2
        , route_add/3
        , route_delete/3
        , route_apply/2
        , subscribe/4
        , unsubscribe/4
        , subscriber_down/3
        , dispatch_batch/2
        , match_routes_batch/2
        , rules_match/4
        ]).

-on_load(init/0).

init() ->
    Dir = case code:priv_dir(emqx) of
              {error, _} -> "priv";
              D -> D
          end,
    erlang:load_nif(filename:join(Dir, "emqx_tm_nif"), 0).

%% new(Device) binds one GPU; new([Device]) one engine over several GPUs (one
%% host trie, an HBM replica on each, per-publish matches dealt over them and
%% batch calls spread over them).  The async pipelines start here.
-spec(new(non_neg_integer() | [non_neg_integer()]) -> {ok, reference()} | {error, term()}).
new(_Devices) -> erlang:nif_error(nif_not_loaded).

%% emqx_trie:insert/1
-spec(insert(reference(), binary()) -> ok | {error, term()}).
insert(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).

%% emqx_trie:delete/1
-spec(delete(reference(), binary()) -> ok | {error, term()}).
delete(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).

%% emqx_trie:lookup/1 -> [#trie_node{}]
-spec(lookup(reference(), binary() | root) -> list()).
lookup(_Engine, _NodeId) -> erlang:nif_error(nif_not_loaded).

%% emqx_trie:empty/0
-spec(empty(reference()) -> boolean()).
empty(_Engine) -> erlang:nif_error(nif_not_loaded).

%% emqx_trie:match/1 (sorted, deduplicated).  The calling process queues its
%% topic and waits for its own reply: every publishing process can have a
%% match in flight, and the engine batches whatever is queued onto the device.
-spec(match(reference(), binary()) -> [binary()] | {error, term()}).
match(Engine, Topic) ->
    Ref = make_ref(),
    case match_async(Engine, Topic, Ref) of
        ok -> receive {emqx_tm_match, Ref, Result} -> Result end;
        {error, _} = Error -> Error
    end.

%% Queue one match; the reply {emqx_tm_match, Ref, [Filter] | {error, Reason}}
%% arrives as a message (runs on a normal scheduler: it only enqueues).
-spec(match_async(reference(), binary(), reference()) -> ok | {error, term()}).
match_async(_Engine, _Topic, _Ref) -> erlang:nif_error(nif_not_loaded).

%% match/1 over a batch of publishes, one device pipeline
-spec(match_batch(reference(), [binary()]) -> [[binary()]]).
match_batch(_Engine, _Topics) -> erlang:nif_error(nif_not_loaded).

%% emqx_topic:match/2 on binaries
-spec(topic_match(binary(), binary()) -> boolean()).
topic_match(_Name, _Filter) -> erlang:nif_error(nif_not_loaded).

%% emqx_router:do_add_route/2 after the mnesia transaction committed.
%% DestId: the caller's id of the route's aggre/1 destination (node(), or the
%% share Group of a {Group, Node} dest), src/emqx_broker.erl:250-261.
-spec(route_add(reference(), binary(), non_neg_integer()) -> ok | {error, term()}).
route_add(_Engine, _Topic, _DestId) -> erlang:nif_error(nif_not_loaded).

%% emqx_router:do_delete_route/2 after the commit.
-spec(route_delete(reference(), binary(), non_neg_integer()) -> ok | {error, term()}).
route_delete(_Engine, _Topic, _DestId) -> erlang:nif_error(nif_not_loaded).

%% Cluster route delta feed: emqx_route table events in order, one call
%% (mnesia replication of remote routes, cleanup_routes/1 on nodedown,
%% shared-subscription {Group, node()} routes).  Absent delete_object = no-op.
-spec(route_apply(reference(), [{write | delete_object, binary(), non_neg_integer()}])
      -> {ok, non_neg_integer()} | {error, term()}).
route_apply(_Engine, _Events) -> erlang:nif_error(nif_not_loaded).

%% Local subscriber bag (emqx_broker do_subscribe/4, do_unsubscribe/4,
%% subscriber_down/1, non-shared): SubId = the caller's id of the subscriber
%% pid, NodeDestId = its id of node() in route_add/3.
-spec(subscribe(reference(), binary(), non_neg_integer(), non_neg_integer()) -> ok | {error, term()}).
subscribe(_Engine, _Topic, _SubId, _NodeDestId) -> erlang:nif_error(nif_not_loaded).

-spec(unsubscribe(reference(), binary(), non_neg_integer(), non_neg_integer()) -> ok | {error, term()}).
unsubscribe(_Engine, _Topic, _SubId, _NodeDestId) -> erlang:nif_error(nif_not_loaded).

-spec(subscriber_down(reference(), non_neg_integer(), non_neg_integer()) -> {ok, non_neg_integer()} | {error, term()}).
subscriber_down(_Engine, _SubId, _NodeDestId) -> erlang:nif_error(nif_not_loaded).

%% emqx_broker:dispatch/2 fan-out for a batch of publishes: per publish the
%% SubIds to deliver to ([] = {error, no_subscribers}).
-spec(dispatch_batch(reference(), [binary()]) -> [[non_neg_integer()]]).
dispatch_batch(_Engine, _Topics) -> erlang:nif_error(nif_not_loaded).

%% aggre(match_routes(Topic)) for a batch of publishes, resolved on the device.
-spec(match_routes_batch(reference(), [binary()]) -> [[{binary(), non_neg_integer()}]]).
match_routes_batch(_Engine, _Topics) -> erlang:nif_error(nif_not_loaded).

%% emqx_topic:match/2 of every name against every rule (ACL: DollarRule = false,
%% rewrite / tracer filters: true); per name the indices of the matching rules.
-spec(rules_match(reference(), [binary()], [binary()], boolean()) -> [[non_neg_integer()]]).
rules_match(_Engine, _Names, _Rules, _DollarRule) -> erlang:nif_error(nif_not_loaded).
