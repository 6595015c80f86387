"""
    SymbolicRegressionMI355X

Julia side of the drop-in: binds `libsr_amd.so` (include/sr_amd.h) with `ccall` and routes
SymbolicRegression's scoring (`_eval_loss`, src/LossFunctions.jl:90-117) through it when the
options are wrapped in `MI355XOptions` — the `AbstractOptions` extension mechanism the reference
documents (src/OptionsStruct.jl:124-175).  Batched entry points (`eval_loss_batch`,
`eval_cost_batch!`) score a whole population per launch for the `Population` / `finalize_costs`
call sites (src/Population.jl:35-61, 182-196).

Not exercised in this repository's CI (no Julia runtime in the build image); the Python mirror in
`../sr_amd` makes the same calls and is what the tests run.
"""
module SymbolicRegressionMI355X

using SymbolicRegression
using SymbolicRegression: AbstractOptions, Dataset, LossFunctionsModule
using DynamicExpressions: AbstractExpressionNode, AbstractExpression, get_tree, get_operators

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
    opsets::Dict{Any,Cint}
    datasets::IdDict{Any,Ptr{Cvoid}}
end

const CONTEXT = Ref{Union{DeviceContext,Nothing}}(nothing)

function context()
    if CONTEXT[] === nothing
        dev = parse(Int, get(ENV, "LOCAL_RANK", "0"))   # one process per GPU
        h = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:sr_init, LIB), Cint, (Cint, Ref{Ptr{Cvoid}}), dev, h))
        CONTEXT[] = DeviceContext(h[], Dict{Any,Cint}(), IdDict{Any,Ptr{Cvoid}}())
    end
    return CONTEXT[]::DeviceContext
end

"""Register `options.operators` once (names as DynamicExpressions prints them)."""
function opset_id(ctx::DeviceContext, operators)
    key = (operators.unaops, operators.binops)
    get!(ctx.opsets, key) do
        un = [string(nameof(f)) for f in operators.unaops]
        bi = [string(nameof(f)) for f in operators.binops]
        id = Ref{Cint}(0)
        rc = ccall((:sr_register_opset, LIB), Cint,
                   (Ptr{Cvoid}, Cint, Ptr{Cstring}, Cint, Ptr{Cstring}, Ref{Cint}),
                   ctx.handle, length(un), un, length(bi), bi, id)
        rc == SR_ERR_UNSUPPORTED_OP && throw(ArgumentError(last_error()))
        check(rc)
        id[]
    end
end

"""Upload `dataset.X` ([nfeatures, n], column-major: exactly the ABI layout), y, weights once."""
function device_dataset(ctx::DeviceContext, dataset::Dataset{T}) where {T}
    get!(ctx.datasets, dataset) do
        X = Matrix{T}(dataset.X)
        out = Ref{Ptr{Cvoid}}(C_NULL)
        w = dataset.weights === nothing ? C_NULL : pointer(Vector{T}(dataset.weights))
        check(ccall((:sr_dataset_upload, LIB), Cint,
                    (Ptr{Cvoid}, Cint, Ptr{T}, Int64, Int64, Ptr{T}, Ptr{Cvoid}, Ref{Ptr{Cvoid}}),
                    ctx.handle, T === Float32 ? SR_DTYPE_F32 : SR_DTYPE_F64, X, size(X, 1), size(X, 2),
                    Vector{T}(dataset.y), w, out))
        out[]
    end
end

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

"""Batched `_eval_loss`: losses::Vector{T} and complete::Vector{Bool} for every tree."""
function eval_loss_batch(trees::AbstractVector, dataset::Dataset{T,L}, options::AbstractOptions;
                         idx::Union{Nothing,AbstractVector{Int}}=nothing) where {T,L}
    ctx = context()
    ops = get_operators(first(trees), options)
    f = flatten(trees, T)
    losses = Vector{T}(undef, length(trees))
    complete = Vector{UInt8}(undef, length(trees))
    rows = idx === nothing ? nothing : Int64.(idx .- 1)   # 0-based SubDataset view
    GC.@preserve f rows begin
        b = SrTreeBatch(length(trees), pointer(f.offsets), pointer(f.degree), pointer(f.op),
                        pointer(f.feature), pointer(f.constant), Ptr{Cvoid}(pointer(f.val)))
        check(ccall((:sr_eval_loss_batch, LIB), Cint,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ref{SrTreeBatch}, Ptr{Int64}, Int64, Cint, Ptr{T}, Ptr{UInt8}),
                    ctx.handle, device_dataset(ctx, dataset), opset_id(ctx, ops), b,
                    rows === nothing ? C_NULL : pointer(rows), rows === nothing ? 0 : length(rows),
                    loss_kind(options), losses, complete))
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
loss_spec(l) = throw(ArgumentError("elementwise_loss $(typeof(l)) stays on the CPU path"))

const LOSS_CODES = Dict{Tuple{Ptr{Cvoid},Int,Float64},Cint}()
function loss_kind(options)
    kind, param = loss_spec(options.elementwise_loss)
    (kind in (0, 1, 3, 9, 10, 11, 12, 14, 15, 16, 17) || (kind == 4 && param == 1.0)) && return Cint(kind)
    ctx = context()
    get!(LOSS_CODES, (ctx.handle, kind, param)) do
        code = Ref{Cint}(0)
        check(ccall((:sr_register_loss, LIB), Cint, (Ptr{Cvoid}, Cint, Cdouble, Ref{Cint}),
                    ctx.handle, kind, param, code))
        code[]
    end
end

"""Batched objective + forward-mode gradient for BFGS (src/ConstantOptimization.jl:126-167):
losses, the gradient of every tree's loss w.r.t. its constants (pre-order, concatenated), complete."""
function eval_grad_batch(trees::AbstractVector, dataset::Dataset{T,L}, options::AbstractOptions) where {T,L}
    ctx = context()
    ops = get_operators(first(trees), options)
    f = flatten(trees, T)
    losses = Vector{T}(undef, length(trees))
    complete = Vector{UInt8}(undef, length(trees))
    grads = zeros(T, count(==(0x01), f.constant) + 1)
    GC.@preserve f begin
        b = SrTreeBatch(length(trees), pointer(f.offsets), pointer(f.degree), pointer(f.op),
                        pointer(f.feature), pointer(f.constant), Ptr{Cvoid}(pointer(f.val)))
        check(ccall((:sr_eval_grad_batch, LIB), Cint,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ref{SrTreeBatch}, Ptr{Int64}, Int64, Cint, Ptr{T}, Ptr{T}, Ptr{UInt8}),
                    ctx.handle, device_dataset(ctx, dataset), opset_id(ctx, ops), b, C_NULL, 0,
                    loss_kind(options), losses, grads, complete))
    end
    return L.(losses), grads[1:end-1], complete .== 0x01
end

"""Batched `eval_cost` (src/LossFunctions.jl:193-209): fills `costs`, `losses` in place."""
function eval_cost_batch!(costs::AbstractVector{L}, losses::AbstractVector{L}, dataset::Dataset{T,L}, members,
                          options::AbstractOptions) where {T,L}
    trees = [m.tree for m in members]
    l, _ = eval_loss_batch(trees, dataset, options)
    for (i, m) in enumerate(members)
        losses[i] = l[i]
        costs[i] = LossFunctionsModule.loss_to_cost(l[i], dataset.use_baseline, dataset.baseline_loss, m, options,
                                                    m.complexity)
    end
    return costs, losses
end

"""Options wrapper selecting the device path: every property forwards to the wrapped options."""
struct MI355XOptions{O<:AbstractOptions} <: AbstractOptions
    base::O
end
Base.getproperty(o::MI355XOptions, s::Symbol) = s === :base ? getfield(o, :base) : getproperty(getfield(o, :base), s)
Base.propertynames(o::MI355XOptions) = propertynames(getfield(o, :base))

# Single-tree scoring (every eval_cost call site) routed through the batch kernel.
function LossFunctionsModule._eval_loss(tree::Union{AbstractExpression{T},AbstractExpressionNode{T}},
                                        dataset::Dataset{T,L}, options::MI355XOptions,
                                        regularization::Bool)::L where {T,L}
    idx = SymbolicRegression.CoreModule.get_indices(dataset)
    full = SymbolicRegression.CoreModule.get_full_dataset(dataset)
    l, _ = eval_loss_batch([tree], full, options; idx=idx)
    loss = l[1]
    if regularization
        loss += LossFunctionsModule.dimensional_regularization(tree, dataset, options)
    end
    return loss
end

end # module
