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
        , match_batch/2
        , topic_match/2
        ]).

-on_load(init/0).

init() ->
    Dir = case code:priv_dir(emqx) of
              {error, _} -> "priv";
              D -> D
          end,
    erlang:load_nif(filename:join(Dir, "emqx_tm_nif"), 0).

-spec(new(non_neg_integer()) -> {ok, reference()} | {error, term()}).
new(_Device) -> erlang:nif_error(nif_not_loaded).

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

%% emqx_trie:match/1 (sorted, deduplicated)
-spec(match(reference(), binary()) -> [binary()]).
match(_Engine, _Topic) -> erlang:nif_error(nif_not_loaded).

%% match/1 over a batch of publishes, one device pipeline
-spec(match_batch(reference(), [binary()]) -> [[binary()]]).
match_batch(_Engine, _Topics) -> erlang:nif_error(nif_not_loaded).

%% emqx_topic:match/2 on binaries
-spec(topic_match(binary(), binary()) -> boolean()).
topic_match(_Name, _Filter) -> erlang:nif_error(nif_not_loaded).
