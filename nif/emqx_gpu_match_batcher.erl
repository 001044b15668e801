%% emqx_gpu_match_batcher — publish batching aggregator in front of the GPU
%% matcher (SURVEY.md §8f rank 2, §7 "Batching a per-message API").
%%
%% The reference publishes one message at a time, in the publisher's own
%% process: emqx_broker:publish/1 (apps/emqx/src/emqx_broker.erl:204-215)
%% traces, counts 'messages.publish', runs the 'message.publish' hook,
%% persists the message, then route(aggre(emqx_router:match_routes(Topic)))
%% (emqx_broker.erl:245-273): a local route dispatches to the topic's
%% subscribers (do_dispatch/2,3, :506-530), a remote one is forwarded
%% (:257-258, forward/4), a shared-group one goes to emqx_shared_sub (:259-260),
%% and an empty route set runs 'message.dropped' + inc_dropped_cnt (:245-248).
%%
%% Here publish/1 keeps all of that in the CALLER's process; only the match
%% moves: the caller asks this gen_server for its topic's groups, the server
%% collects such requests for at most `window_ms` or `max_batch` topics,
%% matches and fans the whole batch out with ONE emqx_gpu_match:fanout_batch/2
%% call, and replies each caller its row: [{Filter, [SubId]}] over every
%% matched route filter (emqx_router:match_routes/1's filters, ascending).  The
%% caller then
%%   * dispatches a filter with local subscribers itself (SubId -> pid through
%%     a read_concurrency ETS table, {deliver, Filter, Msg} per live pid, the
%%     do_dispatch/2 counts and drop hook);
%%   * looks up the other routes of a filter that has any (ETS ?OTHER, kept by
%%     route_add/2 / route_delete/2) with emqx_router:lookup_routes/1 and
%%     forwards / shared-dispatches them as do_route/2 does;
%%   * on {error, _} from the server (no index, a NIF error) routes with
%%     emqx_router:match_routes/1 and emqx_broker:dispatch/2 instead (§8b).
%% So the server process only batches and replies; the 10^9 sends of a hot
%% fan-out (C4) happen in the publishers, as in the reference.
%%
%% Index maintenance is incremental: subscribe/2, unsubscribe/2 (and the
%% monitored death of a subscriber), route_add/2 and route_delete/2 queue ops,
%% and the next flush applies them with ONE emqx_gpu_match:update_subs/2 call
%% (a new snapshot derived from the last; RCU: a NIF call in flight keeps the
%% snapshot it started with).  A filter stays in the index while it has a
%% local subscriber or another destination (route_add).  Wire-up: call
%% route_add/route_delete where emqx_router:do_add_route/2 and
%% do_delete_route/2 (emqx_router.erl:112-125, 164-172) take a destination
%% other than node() -- a remote node, or {Group, Node} of a shared
%% subscription (emqx_shared_sub.erl:308-316) -- and subscribe/unsubscribe
%% where emqx_broker:do_subscribe/4 / do_unsubscribe write the emqx_subscriber
%% bag (emqx_broker.erl:147-165, 445-454) (INTEGRATION.md §4).
%%
%% Built only where erlc / erl_nif.h exist (not in this container); the same
%% logic is mirrored and tested in emqx_amd/batcher.py.
-module(emqx_gpu_match_batcher).
-behaviour(gen_server).

-include_lib("emqx/include/emqx.hrl").

-export([start_link/1, publish/1, publish_batch/1, subscribe/2, unsubscribe/2, route_add/2, route_delete/2,
         stats/0]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2, code_change/3]).

-define(SUBS, emqx_gpu_match_subids).   %% SubId -> Pid
-define(OTHER, emqx_gpu_match_other).   %% Filter -> destinations other than node()
-define(DEFAULT_MAX_BATCH, 4096).
-define(DEFAULT_WINDOW_MS, 1).

-record(st, {index = undefined,
             ops = [] :: [{binary(), non_neg_integer(), atom()}],  %% since the snapshot, newest first
             ids = #{} :: #{pid() => non_neg_integer()},
             filters = #{} :: #{pid() => #{binary() => true}},     %% a subscriber's filters (for its 'DOWN')
             next_id = 0 :: non_neg_integer(),
             pending = [] :: [{gen_server:from(), binary()}],
             n = 0 :: non_neg_integer(),
             timer = undefined,
             max_batch :: pos_integer(),
             window_ms :: non_neg_integer(),
             batches = 0 :: non_neg_integer(),
             messages = 0 :: non_neg_integer(),
             updates = 0 :: non_neg_integer(),
             stale = false :: boolean()}).

%%--------------------------------------------------------------------
%% API
%%--------------------------------------------------------------------

%% Opts: #{max_batch => pos_integer(), window_ms => non_neg_integer()}
start_link(Opts) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Opts, []).

%% emqx_broker:publish/1 with the match batched on the GPU.  Everything but
%% the match runs in the caller, as in the reference (emqx_broker.erl:204-215).
-spec publish(emqx_types:message()) -> emqx_types:publish_result().
publish(Msg) when is_record(Msg, message) ->
    case prepare(Msg) of
        drop -> [];
        {Topic, Delivery} -> route_groups(gen_server:call(?MODULE, {match, Topic}, infinity), Topic, Delivery)
    end.

%% Messages the caller has already collected: one server call for the batch,
%% one publish_result() per message, in order.
-spec publish_batch([emqx_types:message()]) -> [emqx_types:publish_result()].
publish_batch(Msgs) when is_list(Msgs) ->
    Prepared = [prepare(M) || M <- Msgs],
    Topics = [T || {T, _} <- Prepared],
    Rows = case gen_server:call(?MODULE, {match_batch, Topics}, infinity) of
               {ok, Rs} -> [{ok, R} || R <- Rs];
               Err -> [Err || _ <- Topics]
           end,
    results(Prepared, Rows).

%% emqx_broker:do_subscribe/4's subscriber-table write for a plain local
%% subscriber (emqx_broker.erl:147-165): the filter's first holder adds it.
-spec subscribe(binary(), pid()) -> ok.
subscribe(Filter, Pid) when is_binary(Filter), is_pid(Pid) ->
    gen_server:call(?MODULE, {subscribe, Filter, Pid}).

-spec unsubscribe(binary(), pid()) -> ok.
unsubscribe(Filter, Pid) when is_binary(Filter), is_pid(Pid) ->
    gen_server:call(?MODULE, {unsubscribe, Filter, Pid}).

%% A route of Filter to a destination other than node() (do_add_route/2 with
%% a remote node, or {Group, Node} of a shared subscription).
-spec route_add(binary(), term()) -> ok.
route_add(Filter, Dest) when is_binary(Filter) ->
    gen_server:call(?MODULE, {route, Filter, Dest, 1}).

-spec route_delete(binary(), term()) -> ok.
route_delete(Filter, Dest) when is_binary(Filter) ->
    gen_server:call(?MODULE, {route, Filter, Dest, -1}).

stats() -> gen_server:call(?MODULE, stats).

%%--------------------------------------------------------------------
%% caller side: publish/1 around the match, route/2, do_route/2, do_dispatch/2
%%--------------------------------------------------------------------

prepare(Msg) ->
    _ = emqx_trace:publish(Msg),
    emqx_message:is_sys(Msg) orelse emqx_metrics:inc('messages.publish'),
    case emqx_hooks:run_fold('message.publish', [], emqx_message:clean_dup(Msg)) of
        #message{headers = #{allow_publish := false}} -> drop;
        Msg1 = #message{topic = Topic} ->
            emqx_persistent_session:persist_message(Msg1),
            {Topic, #delivery{sender = self(), message = Msg1}}
    end.

results([], []) -> [];
results([drop | Ps], Rows) -> [[] | results(Ps, Rows)];
results([{Topic, D} | Ps], [Row | Rows]) -> [route_groups(Row, Topic, D) | results(Ps, Rows)].

%% The matched filters' routes: local dispatch over the GPU's subscriber ids,
%% lookup_routes/1 only for filters that have other destinations.
route_groups({ok, Groups}, _Topic, Delivery) ->
    Local = [{F, node(), Ids} || {F, Ids = [_ | _]} <- Groups],
    Other = lists:append([[R || R = #route{dest = D} <- emqx_router:lookup_routes(F), D =/= node()]
                          || {F, _} <- Groups, ets:member(?OTHER, F)]),
    route(Local ++ aggre(Other), Delivery);
route_groups({error, _}, Topic, Delivery) ->  %% no usable index: the reference path
    route(aggre(emqx_router:match_routes(Topic)), Delivery).

%% route/2 (emqx_broker.erl:245-253)
route([], #delivery{message = Msg}) ->
    ok = emqx_hooks:run('message.dropped', [Msg, #{node => node()}, no_subscribers]),
    ok = inc_dropped_cnt(Msg),
    [];
route(Routes, Delivery) ->
    lists:foldl(fun(R, Acc) -> [do_route(R, Delivery) | Acc] end, [], Routes).

%% do_route/2 (emqx_broker.erl:255-260); a local route carries its subscriber ids
do_route({To, Node, Ids}, Delivery) ->
    {Node, To, dispatch_ids(To, Ids, Delivery)};
do_route({To, Node}, Delivery) when Node =:= node() ->
    {Node, To, emqx_broker:dispatch(To, Delivery)};
do_route({To, Node}, Delivery) when is_atom(Node) ->
    {Node, To, forward(Node, To, Delivery)};
do_route({To, Group}, Delivery) ->
    {share, To, emqx_shared_sub:dispatch(Group, To, Delivery)}.

%% aggre/1 (emqx_broker.erl:262-273): {To, Node} per node route, one {To, Group} per group
aggre(Routes) ->
    {Nodes, Groups} = lists:foldl(
                        fun(#route{topic = To, dest = {Group, _Node}}, {Ns, Gs}) -> {Ns, [{To, Group} | Gs]};
                           (#route{topic = To, dest = Node}, {Ns, Gs}) -> {[{To, Node} | Ns], Gs}
                        end, {[], []}, Routes),
    Nodes ++ lists:usort(Groups).

forward(Node, To, Delivery) ->
    case emqx:get_config([rpc, mode]) of
        async ->
            true = emqx_broker_proto_v1:forward_async(Node, To, Delivery),
            emqx_metrics:inc('messages.forward');
        sync ->
            case emqx_broker_proto_v1:forward(Node, To, Delivery) of
                {Err, _Reason} when Err =:= badrpc; Err =:= badtcp -> {error, badrpc};
                Result -> emqx_metrics:inc('messages.forward'), Result
            end
    end.

%% dispatch/2 + do_dispatch/2,3 (emqx_broker.erl:296-306, 506-530) over the
%% GPU fan-out's subscriber ids: one {deliver, Filter, Msg} per live pid
dispatch_ids(Filter, Ids, #delivery{message = Msg}) ->
    case emqx:is_running() of
        false -> {error, not_running};
        true ->
            N = lists:foldl(fun(Id, Acc) -> Acc + send(Id, Filter, Msg) end, 0, Ids),
            case N of
                0 ->
                    ok = emqx_hooks:run('message.dropped', [Msg, #{node => node()}, no_subscribers]),
                    ok = inc_dropped_cnt(Msg),
                    {error, no_subscribers};
                _ -> {ok, N}
            end
    end.

send(Id, Filter, Msg) ->
    case ets:lookup(?SUBS, Id) of
        [{_, Pid}] ->
            case erlang:is_process_alive(Pid) of
                true -> Pid ! {deliver, Filter, Msg}, 1;
                false -> 0
            end;
        [] -> 0
    end.

inc_dropped_cnt(Msg) ->
    case emqx_message:is_sys(Msg) of
        true -> ok;
        false ->
            ok = emqx_metrics:inc('messages.dropped'),
            emqx_metrics:inc('messages.dropped.no_subscribers')
    end.

%%--------------------------------------------------------------------
%% gen_server: batching and index maintenance
%%--------------------------------------------------------------------

init(Opts) ->
    _ = ets:new(?SUBS, [named_table, set, protected, {read_concurrency, true}]),
    _ = ets:new(?OTHER, [named_table, set, protected, {read_concurrency, true}]),
    Index = case emqx_gpu_match:load_index([], []) of
                {ok, I} -> I;
                {error, _} -> undefined
            end,
    {ok, #st{index = Index,
             max_batch = maps:get(max_batch, Opts, ?DEFAULT_MAX_BATCH),
             window_ms = maps:get(window_ms, Opts, ?DEFAULT_WINDOW_MS)}}.

handle_call({match, Topic}, From, St = #st{pending = P, n = N, max_batch = Max}) ->
    St1 = St#st{pending = [{From, Topic} | P], n = N + 1},
    case N + 1 >= Max of
        true -> {noreply, flush(St1)};
        false -> {noreply, arm(St1)}
    end;
handle_call({match_batch, Topics}, _From, St) ->
    St1 = refresh(St),
    {reply, match(Topics, St1), count(St1, length(Topics))};
handle_call({subscribe, Filter, Pid}, _From, St) ->
    {Id, St1 = #st{filters = Fs}} = sub_id(Pid, St),
    Mine = maps:get(Pid, Fs, #{}),
    {reply, ok, op({Filter, Id, subscribe}, St1#st{filters = Fs#{Pid => Mine#{Filter => true}}})};
handle_call({unsubscribe, Filter, Pid}, _From, St = #st{ids = I, filters = Fs}) ->
    case maps:find(Pid, I) of
        {ok, Id} ->
            Mine = maps:remove(Filter, maps:get(Pid, Fs, #{})),
            {reply, ok, op({Filter, Id, unsubscribe}, St#st{filters = Fs#{Pid => Mine}})};
        error ->
            {reply, ok, St}
    end;
handle_call({route, _Filter, Dest, _D}, _From, St) when Dest =:= node() ->
    {reply, ok, St};  %% the local route follows the local subscribers (subscribe/2)
handle_call({route, Filter, _Dest, D}, _From, St) ->
    Old = case ets:lookup(?OTHER, Filter) of [{_, C}] -> C; [] -> 0 end,
    New = max(0, Old + D),
    St1 = if
              Old =:= 0, New > 0 -> ets:insert(?OTHER, {Filter, New}), op({Filter, 0, route_add}, St);
              Old > 0, New =:= 0 -> ets:delete(?OTHER, Filter), op({Filter, 0, route_delete}, St);
              true -> ets:insert(?OTHER, {Filter, New}), St
          end,
    {reply, ok, St1};
handle_call(stats, _From, St = #st{batches = B, messages = M, n = N, updates = U, ops = Ops}) ->
    {reply, #{batches => B, messages => M, pending => N, index_updates => U, pending_ops => length(Ops)}, St}.

handle_cast(_Msg, St) -> {noreply, St}.

handle_info(flush_window, St) ->
    {noreply, flush(St#st{timer = undefined})};
handle_info({'DOWN', _Ref, process, Pid, _Reason}, St = #st{ids = I, filters = Fs}) ->
    %% emqx_broker_helper's subscriber_down: every subscription of the pid goes
    case maps:find(Pid, I) of
        {ok, Id} ->
            St1 = lists:foldl(fun(F, S) -> op({F, Id, unsubscribe}, S) end, St, maps:keys(maps:get(Pid, Fs, #{}))),
            true = ets:delete(?SUBS, Id),
            {noreply, St1#st{ids = maps:remove(Pid, I), filters = maps:remove(Pid, Fs)}};
        error ->
            {noreply, St}
    end;
handle_info(_Info, St) -> {noreply, St}.

terminate(_Reason, _St) -> ok.
code_change(_OldVsn, St, _Extra) -> {ok, St}.

%%--------------------------------------------------------------------
%% internals
%%--------------------------------------------------------------------

op(Op, St = #st{ops = Ops}) -> St#st{ops = [Op | Ops]}.

%% the window starts with the first request of a batch
arm(St = #st{timer = undefined, window_ms = W}) ->
    St#st{timer = erlang:send_after(W, self(), flush_window)};
arm(St) -> St.

flush(St = #st{n = 0}) -> St;
flush(St = #st{pending = P, n = N, timer = T}) ->
    _ = case T of undefined -> ok; _ -> erlang:cancel_timer(T) end,
    St1 = refresh(St),
    Batch = lists:reverse(P),
    case match([Topic || {_, Topic} <- Batch], St1) of
        {ok, Rows} -> lists:foreach(fun({{From, _}, Row}) -> gen_server:reply(From, {ok, Row}) end,
                                    lists:zip(Batch, Rows));
        Err -> lists:foreach(fun({From, _}) -> gen_server:reply(From, Err) end, Batch)
    end,
    count(St1#st{pending = [], n = 0, timer = undefined}, N).

match(_Topics, #st{index = undefined}) -> {error, no_index};
match(_Topics, #st{stale = true}) -> {error, stale_index};
match(Topics, #st{index = Index}) ->
    case emqx_gpu_match:fanout_batch(Index, Topics) of
        {error, _} = Err -> Err;
        Rows -> {ok, Rows}
    end.

count(St = #st{batches = B, messages = M}, N) -> St#st{batches = B + 1, messages = M + N}.

sub_id(Pid, St = #st{ids = I, next_id = Next}) ->
    case maps:find(Pid, I) of
        {ok, Id} -> {Id, St};
        error ->
            true = ets:insert(?SUBS, {Next, Pid}),
            _ = erlang:monitor(process, Pid),
            {Next, St#st{ids = I#{Pid => Next}, next_id = Next + 1}}
    end.

%% the queued ops applied to the last snapshot: one update_subs/2 call.  When
%% it fails the ops stay queued (retried at the next flush) and the batch is
%% answered {error, stale_index}: its callers take the reference path, since
%% the old snapshot misses the queued changes.
refresh(St = #st{ops = []}) -> St#st{stale = false};
refresh(St = #st{index = undefined}) -> St;
refresh(St = #st{index = Index, ops = Ops, updates = U}) ->
    case emqx_gpu_match:update_subs(Index, lists:reverse(Ops)) of
        {ok, New} -> St#st{index = New, ops = [], updates = U + 1, stale = false};
        {error, _} -> St#st{stale = true}
    end.
