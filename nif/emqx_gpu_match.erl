%% emqx_gpu_match — Erlang side of the GPU topic-matching NIF (spec + wrapper).
%% Built only where erl_nif.h / erlc exist (not in this container).
%%
%% Drop-in points (reference paths under apps/emqx/src):
%%   match_trie/1 in emqx_router.erl:137-141  -> match_batch/2
%%   match_routes/1 in emqx_router.erl:128-134 -> match_routes_batch/2 (+ lookup_routes/1 per filter)
%%   dispatch/2 in emqx_broker.erl:296-306    -> fanout_batch/2 (index from load_index/2)
%% The publish batching aggregator in front of these is
%% emqx_gpu_match_batcher (publish_batch/1).
%% On {error, _} the wrapper falls back to emqx_trie:match/1 (SURVEY.md §8b).
-module(emqx_gpu_match).

-export([load_index/1, load_index/2, load_index_sharded/1, load_index_sharded/2, update_index/2, update_subs/2,
         match_batch/2, match_routes_batch/2, fanout_batch/2, empty/1, export_index/1, import_index/1]).
-export([match/2]).

-on_load(init/0).

%% LoadInfo: the node's GPUs (application env `gpu_match_devices`, e.g.
%% [0,1,2,3,4,5,6,7]; a single ordinal is one GPU).  With a list, the one NIF
%% context replicates every index to all of them and spreads each batch over
%% them (emqx_gm_opts.n_devices).
init() ->
    Priv = case code:priv_dir(emqx) of {error, _} -> "priv"; D -> D end,
    Devices = application:get_env(emqx, gpu_match_devices, 0),
    erlang:load_nif(filename:join(Priv, "emqx_gpu_match_nif"), Devices).

%% The route filters (emqx_route topics; wildcard ones are the emqx_trie
%% entries) -> an immutable index snapshot in HBM.
-spec load_index([binary()]) -> {ok, reference()} | {error, term()}.
load_index(_Filters) -> erlang:nif_error(nif_not_loaded).

%% Filters with their subscriber ids, one list per filter (the emqx_subscriber
%% bag, emqx_broker.erl:147-165, with its {shard, I} buckets flattened): the
%% index fanout_batch/2 needs.
-spec load_index([binary()], [[non_neg_integer()]]) -> {ok, reference()} | {error, term()}.
load_index(_Filters, _SubIds) -> erlang:nif_error(nif_not_loaded).

%% A route table too large for one GPU: the filters partitioned by first word
%% over the node's GPUs (the NIF context's device list), each topic matched on
%% its one GPU (emqx_gm_index_build_sharded).  Used like any index by the match
%% and fan-out calls; updates and exports of it return {error, _}: rebuild it.
-spec load_index_sharded([binary()]) -> {ok, reference()} | {error, term()}.
load_index_sharded(_Filters) -> erlang:nif_error(nif_not_loaded).

-spec load_index_sharded([binary()], [[non_neg_integer()]]) -> {ok, reference()} | {error, term()}.
load_index_sharded(_Filters, _SubIds) -> erlang:nif_error(nif_not_loaded).

%% Route changes (do_add_route/do_delete_route) as one batch -> a new snapshot;
%% the old one stays valid for readers holding it (emqx_gm_index_update).
%% Any op other than insert | delete is badarg.
-spec update_index(reference(), [{binary(), insert | delete}]) -> {ok, reference()} | {error, term()}.
update_index(_Index, _Ops) -> erlang:nif_error(nif_not_loaded).

%% emqx_gm_index_update_subs on an index from load_index/2: emqx_broker:subscribe/2
%% and unsubscribe/1 in one batch; a filter's first subscriber adds its route, the
%% last one leaving deletes it.  Any other op atom is badarg.
-spec update_subs(reference(), [{binary(), non_neg_integer(), subscribe | unsubscribe}]) ->
          {ok, reference()} | {error, term()}.
update_subs(_Index, _Ops) -> erlang:nif_error(nif_not_loaded).

-spec match_batch(reference(), [binary()]) -> [[binary()]] | {error, term()}.
match_batch(_Index, _Topics) -> erlang:nif_error(nif_not_loaded).

-spec match_routes_batch(reference(), [binary()]) -> [[binary()]] | {error, term()}.
match_routes_batch(_Index, _Topics) -> erlang:nif_error(nif_not_loaded).

%% Per topic: its matched filters, ascending, each with the subscriber ids
%% do_dispatch/2 folds over (a subscriber of two matching filters appears
%% under both: deliveries are a multiset).
-spec fanout_batch(reference(), [binary()]) -> [[{binary(), [non_neg_integer()]}]] | {error, term()}.
fanout_batch(_Index, _Topics) -> erlang:nif_error(nif_not_loaded).

-spec empty(reference()) -> boolean().
empty(_Index) -> erlang:nif_error(nif_not_loaded).

%% The snapshot as one binary (emqx_gm_index_export): what a node joining the
%% cluster imports instead of recompiling the route table -- the reference
%% replicates its routing tables through mria (emqx_router.erl:75-84).
-spec export_index(reference()) -> {ok, binary()} | {error, term()}.
export_index(_Index) -> erlang:nif_error(nif_not_loaded).

%% emqx_gm_index_import on this node's GPU; an image of another table layout
%% (another library build) is {error, _}.
-spec import_index(binary()) -> {ok, reference()} | {error, term()}.
import_index(_Image) -> erlang:nif_error(nif_not_loaded).

%% emqx_trie:match/1 drop-in with fallback.
-spec match(reference(), binary()) -> [binary()].
match(Index, Topic) when is_binary(Topic) ->
    case match_batch(Index, [Topic]) of
        [Row] -> Row;
        {error, _} -> emqx_trie:match(Topic)
    end.
