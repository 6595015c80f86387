"""
    SymbolicRegressionMI355X

Julia side of the drop-in: binds `libsr_amd.so` (include/sr_amd.h) with `ccall` and routes
SymbolicRegression's scoring (`_eval_loss`, src/LossFunctions.jl:90-117) through it when the
options are wrapped in `MI355XOptions` — the `AbstractOptions` extension mechanism the reference
documents (src/OptionsStruct.jl:124-175).

Batching without touching the reference's search code:
* `finalize_costs` (src/Population.jl:182-196) is overridden for `MI355XOptions`: one launch per
  population;
* every other scoring call site (`Population` init src/Population.jl:35-61, `next_generation`
  src/Mutate.jl:270, `crossover_generation` :699-705, constant optimisation, the reload sites) calls
  `_eval_loss` for one tree.  Under `parallelism=:multithreading` the islands run as concurrent
  tasks (src/SearchUtils.jl:289-308) whose calls arrive together: the `BatchScorer` below holds each
  call for a short window and scores everything that arrived in ONE launch, so the islands advance
  in lock-step while each island keeps its serial semantics (it waits for its own result).
* an operator, loss or expression type outside the device catalog keeps the reference's own CPU
  path (`SR_ERR_UNSUPPORTED_OP` -> `_eval_loss(…, options.base, …)`), as INTEGRATION.md states.

Not exercised in this repository's CI (no Julia runtime in the build image); the Python mirror in
`../sr_amd` makes the same calls and is what the tests run.
"""
module SymbolicRegressionMI355X

using SymbolicRegression
using SymbolicRegression: AbstractOptions, Dataset, LossFunctionsModule, PopulationModule, PopMemberModule,
                          SingleIterationModule, ConstantOptimizationModule
using DynamicExpressions: AbstractExpressionNode, AbstractExpression, Expression, Node, get_tree, get_operators,
                          get_scalar_constants, set_scalar_constants!, simplify_tree!, combine_operators

const LIB = get(ENV, "SR_AMD_LIB", joinpath(@__DIR__, "..", "lib", "libsr_amd.so"))

const SR_OK = Cint(0)
const SR_ERR_UNSUPPORTED_OP = Cint(-3)
const SR_DTYPE_F32 = Cint(0)
const SR_DTYPE_F64 = Cint(1)

# Mirrors `sr_tree_batch` (include/sr_amd.h).
struct SrTreeBatch
    n_trees::Int64
    offsets::Ptr{Int64}
    degree::Ptr{UInt8}
    op::Ptr{UInt8}
    feature::Ptr{UInt16}
    constant::Ptr{UInt8}
    val::Ptr{Cvoid}
end

last_error() = unsafe_string(ccall((:sr_last_error, LIB), Cstring, ()))
check(rc) = rc == SR_OK || error("libsr_amd error $(rc): $(last_error())")

mutable struct DeviceContext
    handle::Ptr{Cvoid}
    opsets::Dict{Any,Union{Cint,Nothing}}   # nothing: an operator outside the device catalog
    datasets::IdDict{Any,Ptr{Cvoid}}
    lock::ReentrantLock
end

const CONTEXT = Ref{Union{DeviceContext,Nothing}}(nothing)

function context()
    if CONTEXT[] === nothing
        dev = parse(Int, get(ENV, "LOCAL_RANK", "0"))   # one process per GPU
        h = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:sr_init, LIB), Cint, (Cint, Ref{Ptr{Cvoid}}), dev, h))
        CONTEXT[] = DeviceContext(h[], Dict{Any,Union{Cint,Nothing}}(), IdDict{Any,Ptr{Cvoid}}(), ReentrantLock())
    end
    return CONTEXT[]::DeviceContext
end

"""Register `options.operators` once (names as DynamicExpressions prints them); `nothing` when an
operator is outside the device catalog (the caller keeps the CPU path)."""
function opset_id(ctx::DeviceContext, operators)
    key = (operators.unaops, operators.binops)
    lock(ctx.lock) do
        get!(ctx.opsets, key) do
            un = [string(nameof(f)) for f in operators.unaops]
            bi = [string(nameof(f)) for f in operators.binops]
            id = Ref{Cint}(0)
            rc = ccall((:sr_register_opset, LIB), Cint,
                       (Ptr{Cvoid}, Cint, Ptr{Cstring}, Cint, Ptr{Cstring}, Ref{Cint}),
                       ctx.handle, length(un), un, length(bi), bi, id)
            rc == SR_ERR_UNSUPPORTED_OP && return nothing
            check(rc)
            id[]
        end
    end
end

"""Upload `dataset.X` ([nfeatures, n], column-major: exactly the ABI layout), y, weights once."""
function device_dataset(ctx::DeviceContext, dataset::Dataset{T}) where {T}
    lock(ctx.lock) do
        get!(ctx.datasets, dataset) do
            X = Matrix{T}(dataset.X)
            y = Vector{T}(dataset.y)
            w = dataset.weights === nothing ? nothing : Vector{T}(dataset.weights)
            out = Ref{Ptr{Cvoid}}(C_NULL)
            # every host buffer stays rooted for the whole call (the library copies them)
            GC.@preserve X y w begin
                check(ccall((:sr_dataset_upload, LIB), Cint,
                            (Ptr{Cvoid}, Cint, Ptr{T}, Int64, Int64, Ptr{T}, Ptr{Cvoid}, Ref{Ptr{Cvoid}}),
                            ctx.handle, T === Float32 ? SR_DTYPE_F32 : SR_DTYPE_F64, X, size(X, 1), size(X, 2),
                            y, w === nothing ? C_NULL : Ptr{Cvoid}(pointer(w)), out))
            end
            out[]
        end
    end
end

"""Trees the device evaluates: plain `Expression{T,Node{T,2}}` / `Node` (parametric and template
expressions keep their own evaluators on the CPU)."""
device_tree(t) = t isa Node || (t isa Expression && get_tree(t) isa Node)

"""Pre-order struct-of-arrays of many `Node{T,2}` trees (get_scalar_constants order)."""
function flatten(trees::AbstractVector, ::Type{T}) where {T}
    degree = UInt8[]; op = UInt8[]; feature = UInt16[]; constant = UInt8[]; val = T[]
    offsets = Int64[0]
    for ex in trees
        t = ex isa AbstractExpression ? get_tree(ex) : ex
        stack = Any[t]
        while !isempty(stack)
            n = pop!(stack)
            push!(degree, n.degree)
            if n.degree == 0
                push!(op, 0x00)
                push!(constant, n.constant ? 0x01 : 0x00)
                push!(feature, n.constant ? 0x0000 : n.feature)
                push!(val, n.constant ? n.val : zero(T))
            else
                push!(op, n.op); push!(constant, 0x00); push!(feature, 0x0000); push!(val, zero(T))
                n.degree == 2 && push!(stack, n.r)
                push!(stack, n.l)
            end
        end
        push!(offsets, length(degree))
    end
    return (; offsets, degree, op, feature, constant, val)
end

"""Batched `_eval_loss`: (losses::Vector{L}, complete::Vector{Bool}) for every tree, or `nothing`
when the device cannot evaluate them (operator, loss or expression type outside its catalog: the
caller keeps the reference's CPU path)."""
function eval_loss_batch(trees::AbstractVector, dataset::Dataset{T,L}, options::AbstractOptions;
                         idx::Union{Nothing,AbstractVector{Int}}=nothing) where {T,L}
    isempty(trees) && return (L[], Bool[])
    all(device_tree, trees) || return nothing
    ctx = context()
    oid = opset_id(ctx, get_operators(first(trees), options))
    lk = loss_kind(options)
    (oid === nothing || lk === nothing) && return nothing
    f = flatten(trees, T)
    losses = Vector{T}(undef, length(trees))
    complete = Vector{UInt8}(undef, length(trees))
    rows = idx === nothing ? nothing : Int64.(idx .- 1)   # 0-based SubDataset view
    dsh = device_dataset(ctx, dataset)
    GC.@preserve f rows losses complete begin
        b = SrTreeBatch(length(trees), pointer(f.offsets), pointer(f.degree), pointer(f.op),
                        pointer(f.feature), pointer(f.constant), Ptr{Cvoid}(pointer(f.val)))
        rc = ccall((:sr_eval_loss_batch, LIB), Cint,
                   (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ref{SrTreeBatch}, Ptr{Int64}, Int64, Cint, Ptr{T}, Ptr{UInt8}),
                   ctx.handle, dsh, oid, b, rows === nothing ? C_NULL : pointer(rows),
                   rows === nothing ? 0 : length(rows), lk, losses, complete)
        rc == SR_ERR_UNSUPPORTED_OP && return nothing
        check(rc)
    end
    return L.(losses), complete .== 0x01
end

# Options.elementwise_loss -> (SrLossKind, parameter) (include/sr_amd.h SR_LOSS_*; LossFunctions.jl types as
# src/Options.jl:301-328 lists them); parametric losses are registered once per context.
const LF = SymbolicRegression.LossFunctions
loss_spec(l::LF.L2DistLoss) = (0, 0.0)
loss_spec(l::LF.L1DistLoss) = (1, 0.0)
loss_spec(l::LF.LPDistLoss{P}) where {P} = (2, Float64(P))
loss_spec(l::LF.LogitDistLoss) = (3, 0.0)
loss_spec(l::LF.HuberLoss) = (4, Float64(l.d))
loss_spec(l::LF.L1EpsilonInsLoss) = (5, Float64(l.ε))
loss_spec(l::LF.L2EpsilonInsLoss) = (6, Float64(l.ε))
loss_spec(l::LF.PeriodicLoss) = (7, Float64(2π / l.k))
loss_spec(l::LF.QuantileLoss) = (8, Float64(l.τ))
loss_spec(l::LF.ZeroOneLoss) = (9, 0.0)
loss_spec(l::LF.PerceptronLoss) = (10, 0.0)
loss_spec(l::LF.L1HingeLoss) = (11, 0.0)
loss_spec(l::LF.L2HingeLoss) = (12, 0.0)
loss_spec(l::LF.SmoothedL1HingeLoss) = (13, Float64(l.gamma))
loss_spec(l::LF.ModifiedHuberLoss) = (14, 0.0)
loss_spec(l::LF.L2MarginLoss) = (15, 0.0)
loss_spec(l::LF.ExpLoss) = (16, 0.0)
loss_spec(l::LF.SigmoidLoss) = (17, 0.0)
loss_spec(l::LF.DWDMarginLoss) = (18, Float64(l.q))
loss_spec(l) = nothing  # any other elementwise loss (or a custom function) stays on the CPU path

const LOSS_CODES = Dict{Tuple{Ptr{Cvoid},Int,Float64},Cint}()
function loss_kind(options)
    spec = loss_spec(options.elementwise_loss)
    spec === nothing && return nothing
    kind, param = spec
    (kind in (0, 1, 3, 9, 10, 11, 12, 14, 15, 16, 17) || (kind == 4 && param == 1.0)) && return Cint(kind)
    ctx = context()
    lock(ctx.lock) do; get!(LOSS_CODES, (ctx.handle, kind, param)) do
        code = Ref{Cint}(0)
        check(ccall((:sr_register_loss, LIB), Cint, (Ptr{Cvoid}, Cint, Cdouble, Ref{Cint}),
                    ctx.handle, kind, param, code))
        code[]
    end end
end

"""Batched objective + forward-mode gradient for BFGS (src/ConstantOptimization.jl:126-167):
losses, the gradient of every tree's loss w.r.t. its constants (pre-order, concatenated), complete."""
function eval_grad_batch(trees::AbstractVector, dataset::Dataset{T,L}, options::AbstractOptions) where {T,L}
    all(device_tree, trees) || return nothing
    ctx = context()
    oid = opset_id(ctx, get_operators(first(trees), options))
    lk = loss_kind(options)
    (oid === nothing || lk === nothing) && return nothing
    f = flatten(trees, T)
    losses = Vector{T}(undef, length(trees))
    complete = Vector{UInt8}(undef, length(trees))
    grads = zeros(T, count(==(0x01), f.constant) + 1)
    dsh = device_dataset(ctx, dataset)
    GC.@preserve f losses grads complete begin
        b = SrTreeBatch(length(trees), pointer(f.offsets), pointer(f.degree), pointer(f.op),
                        pointer(f.feature), pointer(f.constant), Ptr{Cvoid}(pointer(f.val)))
        rc = ccall((:sr_eval_grad_batch, LIB), Cint,
                   (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ref{SrTreeBatch}, Ptr{Int64}, Int64, Cint, Ptr{T}, Ptr{T}, Ptr{UInt8}),
                   ctx.handle, dsh, oid, b, C_NULL, 0, lk, losses, grads, complete)
        rc == SR_ERR_UNSUPPORTED_OP && return nothing
        check(rc)
    end
    return L.(losses), grads[1:end-1], complete .== 0x01
end

"""Batched `eval_cost` (src/LossFunctions.jl:193-209): fills `costs`, `losses` in place
(`loss_to_cost` on the host, exactly as the reference).  Falls back to the reference's own
`eval_cost` per member when the device cannot evaluate the trees."""
function eval_cost_batch!(costs::AbstractVector{L}, losses::AbstractVector{L}, dataset::Dataset{T,L}, members,
                          options::AbstractOptions) where {T,L}
    base = options isa MI355XOptions ? options.base : options
    idx = SymbolicRegression.CoreModule.get_indices(dataset)
    full = SymbolicRegression.CoreModule.get_full_dataset(dataset)
    r = eval_loss_batch([m.tree for m in members], full, options; idx=idx)
    for (i, m) in enumerate(members)
        if r === nothing
            costs[i], losses[i] = LossFunctionsModule.eval_cost(dataset, m, base)
        else
            l = r[1][i] + LossFunctionsModule.dimensional_regularization(m.tree, dataset, base)
            losses[i] = l
            costs[i] = LossFunctionsModule.loss_to_cost(l, dataset.use_baseline, dataset.baseline_loss, m, base,
                                                        m.complexity)
        end
    end
    return costs, losses
end

"""Options wrapper selecting the device path: every property forwards to the wrapped options.
`coalesce = true` routes single-tree scoring through the `BatchScorer` (lock-step islands)."""
struct MI355XOptions{O<:AbstractOptions} <: AbstractOptions
    base::O
    coalesce::Bool
end
MI355XOptions(base::AbstractOptions; coalesce::Bool=Threads.nthreads() > 1) = MI355XOptions(base, coalesce)
Base.getproperty(o::MI355XOptions, s::Symbol) =
    s === :base ? getfield(o, :base) : s === :coalesce ? getfield(o, :coalesce) : getproperty(getfield(o, :base), s)
Base.propertynames(o::MI355XOptions) = propertynames(getfield(o, :base))

# ---------------------------------------------------------------- lock-step coalescing
# One request per `_eval_loss` call; the scorer task collects every request that arrives within
# WINDOW_NS of the first (the concurrently running islands reach their next evaluation together),
# groups them by (dataset, row view, options) and scores each group with ONE launch.
struct ScoreRequest
    tree::Any
    dataset::Any          # the full dataset
    idx::Any              # row view (SubDataset indices) or nothing
    options::MI355XOptions
    reply::Channel{Any}   # Vector{L}-element result, or :fallback
end
const QUEUE = Channel{ScoreRequest}(1 << 16)
const SCORER = Ref{Union{Task,Nothing}}(nothing)
const WINDOW_NS = Ref{UInt64}(30_000)
const SCORER_LOCK = ReentrantLock()

function scorer_loop()
    pending = ScoreRequest[]
    while true
        push!(pending, take!(QUEUE))
        t0 = time_ns()
        while time_ns() - t0 < WINDOW_NS[]
            isready(QUEUE) ? push!(pending, take!(QUEUE)) : yield()
        end
        groups = Dict{Any,Vector{ScoreRequest}}()
        for r in pending
            push!(get!(groups, (objectid(r.dataset), r.idx, objectid(r.options.base)), ScoreRequest[]), r)
        end
        for (_, g) in groups
            res = try
                eval_loss_batch([r.tree for r in g], g[1].dataset, g[1].options; idx=g[1].idx)
            catch err
                err
            end
            for (i, r) in enumerate(g)
                put!(r.reply, res === nothing ? :fallback : res isa Exception ? res : res[1][i])
            end
        end
        empty!(pending)
    end
end

function scored_by_batch(tree, full, idx, options::MI355XOptions)
    lock(SCORER_LOCK) do
        if SCORER[] === nothing
            SCORER[] = Threads.@spawn scorer_loop()
        end
    end
    req = ScoreRequest(tree, full, idx, options, Channel{Any}(1))
    put!(QUEUE, req)
    r = take!(req.reply)
    r isa Exception && throw(r)
    return r
end

# Single-tree scoring (every eval_cost call site): the device batch kernel, coalesced across
# concurrently running islands; the reference's own CPU path when the device cannot evaluate it.
function LossFunctionsModule._eval_loss(tree::Union{AbstractExpression{T},AbstractExpressionNode{T}},
                                        dataset::Dataset{T,L}, options::MI355XOptions,
                                        regularization::Bool)::L where {T,L}
    idx = SymbolicRegression.CoreModule.get_indices(dataset)
    full = SymbolicRegression.CoreModule.get_full_dataset(dataset)
    loss = if options.coalesce
        scored_by_batch(tree, full, idx, options)
    else
        r = eval_loss_batch([tree], full, options; idx=idx)
        r === nothing ? :fallback : r[1][1]
    end
    loss === :fallback && return LossFunctionsModule._eval_loss(tree, dataset, options.base, regularization)
    if regularization
        loss += LossFunctionsModule.dimensional_regularization(tree, dataset, options)
    end
    return loss
end

# ---------------------------------------------------------------- batched constant optimisation
const Optim = ConstantOptimizationModule.Optim
const LineSearches = ConstantOptimizationModule.LineSearches

"""The device optimiser is the reference's DEFAULT one only: `Optim.BFGS(; linesearch=LineSearches.
BackTracking())` (src/Options.jl:613-615), with Newton for a single constant as `optimize_constants`
itself chooses (src/ConstantOptimization.jl:38-56).  Returns `(iterations, f_calls_limit)` from
`options.optimizer_options` (the `Optim.Options` built at src/Options.jl:988-997) when the device can
run it, or `nothing`: any other `optimizer_algorithm` (`NelderMead`, accepted at Options.jl:738-746),
another line search or BackTracking setting (incl. `iterations`, `maxstep`), a non-identity initial
inverse Hessian, an `initial_stepnorm`, a manifold other than `Flat`, or Optim options
beyond `iterations` / `f_calls_limit` at non-default values — the caller then keeps the reference's
per-member `optimize_constants` (INTEGRATION.md §4)."""
function device_optimizer(options)
    alg = options.optimizer_algorithm
    alg isa Optim.BFGS || return nothing
    ls = getfield(alg, :linesearch!)
    ls isa LineSearches.BackTracking || return nothing
    (ls.c_1 == 1e-4 && ls.ρ_hi == 0.5 && ls.ρ_lo == 0.1 && ls.order == 3) || return nothing
    # (BackTracking's remaining fields and BFGS's step norm / manifold at their defaults too: the device
    #  optimiser implements exactly that configuration — ADVICE r5)
    (ls.iterations == 1000 && isinf(ls.maxstep)) || return nothing
    getfield(alg, :initial_invH) === nothing || return nothing
    getfield(alg, :initial_stepnorm) === nothing || return nothing
    getfield(alg, :manifold) isa Optim.Flat || return nothing
    getfield(alg, :alphaguess!) isa LineSearches.InitialStatic || return nothing
    o = options.optimizer_options
    # the device's stopping rules: g_abstol 1e-8 (Optim's default), iterations, f_calls_limit
    (o.g_abstol == 1e-8 && o.x_abstol == 0 && o.f_abstol == 0 && o.f_reltol == 0 && o.x_reltol == 0 &&
     o.callback === nothing && isnan(o.time_limit)) || return nothing
    return (Cint(o.iterations), Int64(o.f_calls_limit))
end

"""Batched `optimize_constants` (src/ConstantOptimization.jl:29-116) of `members` on `dataset` (a full
dataset or a SubDataset view): ONE `sr_optimize_constants_batch` call runs the reference's algorithm
for every member in lock-step on the device (BFGS + BackTracking, Newton for one constant, from the
constants and `optimizer_nrestarts` perturbed starts, the minimum adopted only if it beats the start;
each line-search round one batched loss launch, each gradient one forward-mode launch).  Updates the
improved members' constants, loss, cost and birth like `_optimize_constants_inner` and returns their
`num_evals` (objective calls x dataset fraction, +1 per improved member), or `nothing` when the device
cannot take these trees or this optimiser (`device_optimizer`; the caller then keeps the reference's
per-member path)."""
function optimize_constants_batch!(dataset::Dataset{T,L}, members::AbstractVector, options::MI355XOptions
                                   ) where {T,L}
    isempty(members) && return Float64[]
    limits = device_optimizer(options)
    limits === nothing && return nothing
    iterations, f_calls_limit = limits
    trees = [m.tree for m in members]
    all(device_tree, trees) || return nothing
    ctx = context()
    oid = opset_id(ctx, get_operators(first(trees), options))
    lk = loss_kind(options)
    (oid === nothing || lk === nothing) && return nothing
    idx = SymbolicRegression.CoreModule.get_indices(dataset)
    full = SymbolicRegression.CoreModule.get_full_dataset(dataset)
    f = flatten(trees, T)
    n = length(trees)
    consts = Vector{T}(undef, max(1, count(==(0x01), f.constant)))
    losses = Vector{T}(undef, n)
    improved = Vector{UInt8}(undef, n)
    f_calls = Vector{Int64}(undef, n)
    rows = idx === nothing ? nothing : Int64.(idx .- 1)
    dsh = device_dataset(ctx, full)
    seed = rand(UInt64)   # the restart draws (x0 .* (1 + eps/2), eps ~ randn) come from this stream
    GC.@preserve f rows consts losses improved f_calls begin
        b = SrTreeBatch(n, pointer(f.offsets), pointer(f.degree), pointer(f.op), pointer(f.feature),
                        pointer(f.constant), Ptr{Cvoid}(pointer(f.val)))
        rc = ccall((:sr_optimize_constants_batch, LIB), Cint,
                   (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ref{SrTreeBatch}, Ptr{Int64}, Int64, Cint, Cint, Int64, Cint,
                    UInt64, Ptr{T}, Ptr{T}, Ptr{UInt8}, Ptr{Int64}),
                   ctx.handle, dsh, oid, b, rows === nothing ? C_NULL : pointer(rows),
                   rows === nothing ? 0 : length(rows), lk, iterations, f_calls_limit,
                   options.optimizer_nrestarts, seed, consts, losses, improved, f_calls)
        rc == SR_ERR_UNSUPPORTED_OP && return nothing
        check(rc)
    end
    base = options.base
    frac = SymbolicRegression.CoreModule.dataset_fraction(dataset)
    num_evals = zeros(Float64, n)
    at = 0
    for (k, m) in enumerate(members)
        x0, refs = get_scalar_constants(m.tree)   # pre-order: the order the library returned them in
        nk = length(x0)
        num_evals[k] = f_calls[k] * frac
        if improved[k] == 0x01
            set_scalar_constants!(m.tree, consts[at+1:at+nk], refs)
            m.loss = L(losses[k]) + LossFunctionsModule.dimensional_regularization(m.tree, dataset, base)
            m.cost = LossFunctionsModule.loss_to_cost(m.loss, dataset.use_baseline, dataset.baseline_loss, m, base)
            m.birth = SymbolicRegression.UtilsModule.get_birth_order(; deterministic=base.deterministic)
            num_evals[k] += frac
        end
        at += nk
    end
    return num_evals
end

# `optimize_and_simplify_population` (src/SingleIteration.jl:68-139): simplification per member as the
# reference, then the selected members' constants optimised in ONE batched device call instead of one
# Optim run per member (:79-92), then `finalize_costs` and the new references.  With the recorder on
# (or trees the device cannot take) the reference's own function runs.
function SingleIterationModule.optimize_and_simplify_population(
    dataset::D, pop::P, options::MI355XOptions, curmaxsize::Int, record::SymbolicRegression.RecordType
)::Tuple{P,Float64} where {T,L,D<:Dataset{T,L},P<:PopulationModule.Population{T,L}}
    base = options.base
    base.use_recorder && return SingleIterationModule.optimize_and_simplify_population(dataset, pop, base,
                                                                                       curmaxsize, record)
    do_optimization = rand(pop.n) .< options.optimizer_probability
    batched_dataset = options.batching ? SymbolicRegression.CoreModule.batch(dataset, options.batch_size) : dataset
    if options.should_simplify
        for m in pop.members
            tree = simplify_tree!(m.tree, options.operators)
            m.tree = combine_operators(tree, options.operators)
        end
    end
    num_evals = 0.0
    if options.should_optimize_constants
        sel = [m for (m, d) in zip(pop.members, do_optimization) if d &&
               ConstantOptimizationModule.count_constants_for_optimization(m.tree) > 0]
        ev = optimize_constants_batch!(batched_dataset, sel, options)
        if ev === nothing  # the reference's per-member optimiser
            for m in sel
                _, e = ConstantOptimizationModule.optimize_constants(batched_dataset, m, base)
                num_evals += e
            end
        else
            num_evals += sum(ev; init=0.0)
        end
    end
    pop, tmp_num_evals = PopulationModule.finalize_costs(dataset, pop, options)
    num_evals += tmp_num_evals
    for m in pop.members
        old_ref = m.ref
        m.parent = old_ref
        m.ref = PopMemberModule.generate_reference()
    end
    return (pop, num_evals)
end

# `finalize_costs` (src/Population.jl:182-196): one launch for the whole population.
function PopulationModule.finalize_costs(dataset::Dataset{T,L}, pop::P, options::MI355XOptions
                                         )::Tuple{P,Float64} where {T,L,P<:PopulationModule.Population{T,L}}
    options.batching || return (pop, 0.0)
    costs = Vector{L}(undef, pop.n)
    losses = Vector{L}(undef, pop.n)
    eval_cost_batch!(costs, losses, dataset, pop.members, options)
    for (m, c, l) in zip(pop.members, costs, losses)
        m.cost = c
        m.loss = l
    end
    return (pop, Float64(pop.n))
end

end # module
