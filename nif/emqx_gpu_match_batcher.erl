%% emqx_gpu_match_batcher — publish batching aggregator in front of the GPU
%% matcher (SURVEY.md §8f rank 2, §7 "Batching a per-message API").
%%
%% The reference publishes one message at a time, in the publisher's own
%% process: emqx_broker:publish/1 (apps/emqx/src/emqx_broker.erl:204-215) ->
%% emqx_router:match_routes/1 -> route/2 -> dispatch/2 -> do_dispatch/2,3
%% (emqx_broker.erl:245-260, 296-322, 506-530).  A GPU call pays off only
%% over many topics, so this gen_server collects published messages for at
%% most `window_ms` or `max_batch` messages, whichever comes first, matches
%% and fans the whole batch out with ONE emqx_gpu_match:fanout_batch/2 call,
%% maps the subscriber ids back to pids and sends {deliver, Filter, Msg}
%% exactly as do_dispatch/3 does.  Each caller of publish/1 gets its own
%% publish_result() back once its batch is dispatched: the latency of a
%% publish is bounded by the window plus one batch (DESIGN.md "Host path").
%%
%% Subscribers are kept as dense ids (the GPU index carries u32 ids, not
%% pids): subscribe/2 assigns one per pid, the {Filter -> [SubId]} table is
%% what load_index/2 takes, and a changed table becomes a new index snapshot
%% at the next flush (RCU: a batch in flight keeps the snapshot it started
%% with).  Scope: local subscribers (the route dest node()); remote and
%% shared-group routes keep going through emqx_broker:route/2.
%% On {error, _} from the NIF every message of the batch falls back to
%% emqx_broker:publish/1 (SURVEY.md §8b).
%%
%% Built only where erlc / erl_nif.h exist (not in this container); the same
%% window logic is mirrored and tested in emqx_amd/batcher.py.
-module(emqx_gpu_match_batcher).
-behaviour(gen_server).

-include_lib("emqx/include/emqx.hrl").

-export([start_link/1, publish/1, publish_batch/1, subscribe/2, unsubscribe/2, stats/0]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2, code_change/3]).

-define(SUBS, emqx_gpu_match_subids).  %% SubId -> Pid
-define(DEFAULT_MAX_BATCH, 4096).
-define(DEFAULT_WINDOW_MS, 1).

-record(st, {index = undefined,
             dirty = true,
             filters = #{} :: #{binary() => [non_neg_integer()]},
             ids = #{} :: #{pid() => non_neg_integer()},
             next_id = 0 :: non_neg_integer(),
             pending = [] :: [{gen_server:from(), emqx_types:message()}],
             n = 0 :: non_neg_integer(),
             timer = undefined,
             max_batch :: pos_integer(),
             window_ms :: non_neg_integer(),
             batches = 0 :: non_neg_integer(),
             messages = 0 :: non_neg_integer()}).

%%--------------------------------------------------------------------
%% API
%%--------------------------------------------------------------------

%% Opts: #{max_batch => pos_integer(), window_ms => non_neg_integer()}
start_link(Opts) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Opts, []).

%% emqx_broker:publish/1 through the aggregator.  The 'message.publish' hook
%% runs in the caller, as in the reference (emqx_broker.erl:207-212); the
%% call returns when the batch holding the message has been dispatched.
-spec publish(emqx_types:message()) -> emqx_types:publish_result().
publish(Msg) when is_record(Msg, message) ->
    case emqx_hooks:run_fold('message.publish', [], emqx_message:clean_dup(Msg)) of
        #message{headers = #{allow_publish := false}} -> [];
        Msg1 -> gen_server:call(?MODULE, {publish, Msg1}, infinity)
    end.

%% A batch the caller has already collected: dispatched at once, one result
%% per message, in order.
-spec publish_batch([emqx_types:message()]) -> [emqx_types:publish_result()].
publish_batch(Msgs) when is_list(Msgs) ->
    gen_server:call(?MODULE, {publish_batch, Msgs}, infinity).

%% emqx_broker:subscribe/3's subscriber-table write (emqx_broker.erl:147-165).
-spec subscribe(binary(), pid()) -> ok.
subscribe(Filter, Pid) when is_binary(Filter), is_pid(Pid) ->
    gen_server:call(?MODULE, {subscribe, Filter, Pid}).

-spec unsubscribe(binary(), pid()) -> ok.
unsubscribe(Filter, Pid) when is_binary(Filter), is_pid(Pid) ->
    gen_server:call(?MODULE, {unsubscribe, Filter, Pid}).

stats() -> gen_server:call(?MODULE, stats).

%%--------------------------------------------------------------------
%% gen_server
%%--------------------------------------------------------------------

init(Opts) ->
    _ = ets:new(?SUBS, [named_table, set, protected, {read_concurrency, true}]),
    {ok, #st{max_batch = maps:get(max_batch, Opts, ?DEFAULT_MAX_BATCH),
             window_ms = maps:get(window_ms, Opts, ?DEFAULT_WINDOW_MS)}}.

handle_call({publish, Msg}, From, St = #st{pending = P, n = N, max_batch = Max}) ->
    St1 = St#st{pending = [{From, Msg} | P], n = N + 1},
    case N + 1 >= Max of
        true -> {noreply, flush(St1)};
        false -> {noreply, arm(St1)}
    end;
handle_call({publish_batch, Msgs}, _From, St) ->
    St1 = refresh(St),
    {reply, dispatch(Msgs, St1#st.index), count(St1, length(Msgs))};
handle_call({subscribe, Filter, Pid}, _From, St = #st{filters = F}) ->
    {Id, St1} = sub_id(Pid, St),
    Ids = maps:get(Filter, F, []),
    case lists:member(Id, Ids) of
        true -> {reply, ok, St1};
        false -> {reply, ok, St1#st{filters = F#{Filter => Ids ++ [Id]}, dirty = true}}
    end;
handle_call({unsubscribe, Filter, Pid}, _From, St = #st{filters = F, ids = I}) ->
    case {maps:find(Pid, I), maps:find(Filter, F)} of
        {{ok, Id}, {ok, Ids}} ->
            F1 = case lists:delete(Id, Ids) of
                     [] -> maps:remove(Filter, F);
                     Rest -> F#{Filter => Rest}
                 end,
            {reply, ok, St#st{filters = F1, dirty = true}};
        _ ->
            {reply, ok, St}
    end;
handle_call(stats, _From, St = #st{batches = B, messages = M, n = N}) ->
    {reply, #{batches => B, messages => M, pending => N}, St}.

handle_cast(_Msg, St) -> {noreply, St}.

handle_info(flush_window, St) ->
    {noreply, flush(St#st{timer = undefined})};
handle_info(_Info, St) -> {noreply, St}.

terminate(_Reason, _St) -> ok.
code_change(_OldVsn, St, _Extra) -> {ok, St}.

%%--------------------------------------------------------------------
%% internals
%%--------------------------------------------------------------------

%% the window starts with the first message of a batch
arm(St = #st{timer = undefined, window_ms = W}) ->
    St#st{timer = erlang:send_after(W, self(), flush_window)};
arm(St) -> St.

flush(St = #st{n = 0}) -> St;
flush(St = #st{pending = P, n = N, timer = T}) ->
    _ = case T of undefined -> ok; _ -> erlang:cancel_timer(T) end,
    St1 = refresh(St),
    Batch = lists:reverse(P),
    Results = dispatch([M || {_, M} <- Batch], St1#st.index),
    lists:foreach(fun({{From, _}, R}) -> gen_server:reply(From, R) end, lists:zip(Batch, Results)),
    count(St1#st{pending = [], n = 0, timer = undefined}, N).

count(St = #st{batches = B, messages = M}, N) -> St#st{batches = B + 1, messages = M + N}.

sub_id(Pid, St = #st{ids = I, next_id = Next}) ->
    case maps:find(Pid, I) of
        {ok, Id} -> {Id, St};
        error ->
            true = ets:insert(?SUBS, {Next, Pid}),
            {Next, St#st{ids = I#{Pid => Next}, next_id = Next + 1}}
    end.

%% a new snapshot when the subscriber table changed since the last one
refresh(St = #st{dirty = false}) -> St;
refresh(St = #st{filters = F}) ->
    {Filters, SubIds} = lists:unzip(maps:to_list(F)),
    case emqx_gpu_match:load_index(Filters, SubIds) of
        {ok, Index} -> St#st{index = Index, dirty = false};
        {error, _} -> St#st{index = undefined}
    end.

dispatch(Msgs, undefined) ->
    [emqx_broker:publish(M) || M <- Msgs];
dispatch(Msgs, Index) ->
    case emqx_gpu_match:fanout_batch(Index, [emqx_message:topic(M) || M <- Msgs]) of
        {error, _} -> dispatch(Msgs, undefined);
        Rows -> lists:zipwith(fun deliver/2, Msgs, Rows)
    end.

%% route/2 for one message over its matched filters (emqx_broker.erl:245-260)
deliver(_Msg, []) -> [];  %% no route: counted as dropped by the caller's metrics, as route([], _)
deliver(Msg, Groups) ->
    [{node(), Filter, dispatch_group(Filter, SubIds, Msg)} || {Filter, SubIds} <- Groups].

%% do_dispatch/2,3 (emqx_broker.erl:506-530): one {deliver, Filter, Msg} per live subscriber
dispatch_group(Filter, SubIds, Msg) ->
    N = lists:foldl(
          fun(Id, Acc) ->
                  case ets:lookup(?SUBS, Id) of
                      [{_, Pid}] ->
                          case erlang:is_process_alive(Pid) of
                              true -> Pid ! {deliver, Filter, Msg}, Acc + 1;
                              false -> Acc
                          end;
                      [] -> Acc
                  end
          end, 0, SubIds),
    case N of
        0 -> {error, no_subscribers};
        _ -> {ok, N}
    end.
