"""Universe / UniverseGAN with the MI355X ``enhance()``.

Mirrors networks/universe/universe.py (Universe, :44-386) and
networks/universe/universe_gan.py (UniverseGAN, :62-151) for inference: same
constructor signature (training-only arguments accepted and ignored), same
parameter tree and ``model_parameters()`` order (the torch_ema positional
contract), same ``enhance`` signature and type hints (the CLI derives its
arguments from them, inference_utils/signature_to_parser.py:26-66).

``enhance`` records the whole sampler for a (batch, length, options) shape once
(plan.EnhancePlan) and replays it as a hipGraph: conditioner, loop-invariant
signal-conditioning projections, every FiLM vector of every step, the N score
network passes with the EDM wrapper and the sampler update fused into the
output convolution, then crop / keep_rms / peak normalisation.  Noise is drawn
with ``torch.randn(..., generator=rng)`` on the device in the reference's order
(x0, then one z per step), so a run is bit-comparable in its noise to the
reference on the same device and generator.
"""
import collections
import itertools
import math
import os
from typing import Optional

import torch
from torch import nn

from ... import _lib as L
from .blocks import PReLU_Conv
from .condition import ConditionerNetwork
from .score import ScoreNetwork


class AttrDict(dict):
    """dict with attribute access (stands in for the reference's DictConfig)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def _as_attr(x):
    if isinstance(x, dict):
        return AttrDict({k: _as_attr(v) for k, v in x.items()})
    return x


def _strip_target(cfg):
    return {k: v for k, v in dict(cfg).items() if k != "_target_"}


class Universe(nn.Module):
    def __init__(self, fs, normalization_norm, score_model, condition_model, diffusion,
                 losses=None, training=None, validation=None, optimizer=None, scheduler=None,
                 grad_clipper=None, transform=None, normalization_kwargs=None,
                 with_noise_target=False, detach_cond=False, edm=None):
        super().__init__()
        if transform is not None:
            raise NotImplementedError("only the identity transform is on the target configs")
        if normalization_norm not in (2, "2"):
            raise NotImplementedError(f"normalization_norm={normalization_norm}")
        self.fs = fs
        self.normalization_norm = normalization_norm
        self.normalization_kwargs = dict(normalization_kwargs or {})
        self.diff_kwargs = _as_attr(dict(diffusion))
        self.losses_kwargs = losses or {}
        self._score_cfg = _strip_target(score_model)
        self._cond_cfg = _strip_target(condition_model)
        self.edm_kwargs = _as_attr(dict(edm)) if edm is not None else None
        self.with_edm = edm is not None
        if self.with_edm:
            self._edm_model = ScoreNetwork(**self._score_cfg)
        else:
            self.score_model = ScoreNetwork(**self._score_cfg)
        self.condition_model = ConditionerNetwork(**self._cond_cfg)
        rate_factors = self._score_cfg.get("rate_factors", [2, 4, 4, 5])
        self.n_channels = self._score_cfg.get("n_channels", 32)
        self.n_stages = len(rate_factors)
        self.latent_n_channels = 2**self.n_stages * self.n_channels
        self.tot_ds = math.prod(rate_factors)
        self.init_losses(score_model, condition_model, self.losses_kwargs, training)
        self.ema = None  # EMA weights are applied at load time (inference only)
        self._engine = None
        self._plans = collections.OrderedDict()   # LRU of recorded plans, see _plan()
        self._inflight = set()   # plan keys submitted by enhance_many and not yet checked
        self._conv_prec = None   # None: OUHIP_CONV_PREC; 0 after a range error no exponent widening fixed
        self.range_fallbacks = 0   # enhance()/enhance_many() calls rerun with f32 operands
        self.range_widenings = 0   # reruns after widening the staging exponents of named layers

    def init_losses(self, score_model, condition_model, losses, training):
        """Training losses are out of scope; nothing to build for Universe."""

    def model_parameters(self):
        """universe.py:134-137: the EMA's positional parameter order."""
        return itertools.chain(self.get_score_model().parameters(), self.condition_model.parameters())

    def get_score_model(self):
        return self._edm_model if self.with_edm else self.score_model

    def aux_to_wav(self, y_aux):
        return y_aux

    # ------------------------------------------------------------------ engine
    def _model_cfg(self):
        return {
            "fs": self.fs,
            "normalization_kwargs": self.normalization_kwargs,
            "edm": dict(self.edm_kwargs) if self.edm_kwargs is not None else None,
            "score_model": self.get_score_model().config,
            "condition_model": self.condition_model.config,
            "diffusion": dict(self.diff_kwargs),
        }

    def _get_engine(self):
        from ...engine import Engine

        dev = next(self.parameters()).device
        if self._engine is None or self._engine.device != dev:
            self._engine = Engine(self._model_cfg(), self.state_dict(), dev, conv_prec=self._conv_prec)
            self._plans = collections.OrderedDict()
        return self._engine

    def _plan(self, key, make):
        """The recorded plan for a (batch, length, options) key.  Plans are
        kept in an LRU of OUHIP_MAX_PLANS (default 8) entries: a stream of clips
        of many lengths (the CLI over a folder) records one plan per length and
        evicts the least recently used, whose buffers return to the caching
        allocator for the next plan.  Tiles are tuned once per layer geometry
        (engine.ConvTuner reuses them across lengths), so recording a plan for a
        new length launches nothing but the graph capture."""
        plan = self._plans.get(key)
        if plan is not None:
            self._plans.move_to_end(key)
            return plan
        cap = max(1, int(os.environ.get("OUHIP_MAX_PLANS", "8")))
        # plans enhance_many has queued and not yet synchronised are pinned:
        # their kernels may still read the buffers an eviction would free
        while len(self._plans) >= cap:
            victim = next((k for k in self._plans if k not in self._inflight), None)
            if victim is None:
                break
            del self._plans[victim]
        plan = self._plans[key] = make()
        return plan

    def _arena_plan(self, key, slot, build):
        """_plan() for an EnhancePlan recorded onto the engine's arena of
        ``slot`` (engine.Arena): ``build(arena)`` records the plan.  An arena
        that is too small is replaced by one of at least twice the size; the
        plans recorded on the old one are dropped (re-recorded when used)."""
        from ... import engine as E

        eng = self._get_engine()
        if os.environ.get("OUHIP_ARENA", "1") == "0":
            return self._plan(key, lambda: build(None))
        arenas = eng.__dict__.setdefault("arenas", {})

        def make():
            while True:
                ar = arenas.get(slot)
                if ar is None:
                    ar = arenas[slot] = E.Arena(eng.device, 64 << 20)
                try:
                    return build(ar)
                except E.ArenaFull as e:
                    size = max(2 * ar.nbytes, int(e.args[0] * 1.5))
                    old = [k for k, p in self._plans.items() if getattr(p, "arena", None) is ar]
                    if any(k in self._inflight for k in old):
                        # plans of this slot are still queued on its stream:
                        # their kernels read the arena being replaced
                        torch.cuda.synchronize(eng.device)
                        self._inflight.clear()
                    for k in old:
                        del self._plans[k]
                    arenas[slot] = None
                    del ar
                    arenas[slot] = E.Arena(eng.device, size)

        return self._plan(key, make)

    def invalidate(self):
        """Drop the packed device weights (call after changing parameters)."""
        self._engine, self._plans = None, collections.OrderedDict()
        self._inflight = set()

    def _apply(self, fn, *args, **kwargs):
        self.invalidate()
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self.invalidate()
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def train(self, mode=True, no_ema=False):
        return super().train(mode)

    def eval(self, no_ema=False):
        return self.train(False)

    def forward(self, xt, sigma, cond):
        return self.score_model_call(xt, sigma, cond)

    def score_model_call(self, x, sigma, cond):
        """score_model / _edm_score_wrapper (universe.py:197-209) on the device."""
        if not self.with_edm:
            return self.score_model(x, sigma, cond)
        from ...plan import edm_weights  # noqa: F401  (documented coefficients)

        lvl = self.edm_kwargs.get("data_level_db", self.normalization_kwargs.get("level_db", 0.0))
        sigma_data = 10.0 ** (lvl / 20.0)
        sigma_norm = (sigma**2 + sigma_data**2) ** 0.5
        w_in = (1.0 / sigma_norm)[:, None, None]
        w_skip = (sigma_data**2 / (sigma**2 + sigma_data**2))[:, None, None]
        w_out = (sigma * sigma_data / sigma_norm)[:, None, None]
        net = self._edm_model(w_in * x, self.edm_kwargs["noise"] * sigma, cond)
        est = w_skip * x + w_out * net
        return (est - x) / sigma[:, None, None] ** 2

    # ------------------------------------------------------------------ noise
    def noise_shapes(self, mix_shape, n_steps: Optional[int] = None, target=None, use_aux_signal=False,
                     ensemble=None, warm_start=None, **_):
        """The shapes of the ``torch.randn(..., generator=rng)`` draws one
        ``enhance(mix, ...)`` makes, in draw order (universe.py:39-41,322-343:
        x0, then one z per intermediate step; the known-answer mode also draws
        the score noise of every step, :278-298).  Drawing and discarding
        these advances ``rng`` exactly as that enhance would (bin/enhance.py
        keeps a multi-rank run's noise assignment equal to the 1-rank run's)."""
        if n_steps is None:
            n_steps = self.diff_kwargs.n_steps
        shape = tuple(mix_shape)
        if len(shape) == 1:
            shape = (1, 1) + shape
        elif len(shape) == 2:
            shape = (shape[0], 1, shape[1])
        B, T = shape[0] * (ensemble or 1), shape[-1]
        Tp = T + self.tot_ds - T % self.tot_ds
        if target is not None:
            return [(B, 1, Tp)] * (2 * int(n_steps))
        if use_aux_signal:
            return []
        n_start = 0 if warm_start is None else int(warm_start)
        return [(B, 1, Tp)] * (1 + (int(n_steps) - 1 - n_start))

    def skip_noise(self, mix_shape, rng, **enhance_kwargs):
        """Advance ``rng`` past the noise of an ``enhance`` of ``mix_shape``
        without running it (the draws are made and discarded)."""
        if rng is None:
            return
        for shp in self.noise_shapes(mix_shape, **enhance_kwargs):
            torch.randn(shp, generator=rng, device=rng.device, dtype=torch.float32)

    # ------------------------------------------------------------------ enhance
    def enhance(
        self,
        mix,
        n_steps: Optional[int] = None,
        epsilon: Optional[float] = None,
        target: Optional[torch.Tensor] = None,
        fake_score_snr: Optional[float] = None,
        rng: Optional[torch.Generator] = None,
        use_aux_signal: Optional[bool] = False,
        keep_rms: Optional[bool] = False,
        ensemble: Optional[int] = None,
        ensemble_stat: Optional[str] = "median",
        warm_start: Optional[int] = None,
    ) -> torch.Tensor:
        """Reverse-diffusion enhancement (universe.py:231-375)."""
        from ...plan import EnhancePlan

        if epsilon is None:
            epsilon = self.diff_kwargs.epsilon
        if n_steps is None:
            n_steps = self.diff_kwargs.n_steps
        x_ndim = mix.ndim
        if x_ndim == 1:
            mix = mix[None, None, :]
        elif x_ndim == 2:
            mix = mix[:, None, :]
        elif x_ndim > 3:
            raise ValueError("The input should have at most 3 dimensions")
        if ensemble_stat not in ("mean", "median", "signal_median") and ensemble is not None:
            raise NotImplementedError()
        if target is not None:
            x = self._enhance_fake_score(mix, n_steps, epsilon, target, fake_score_snr, rng,
                                         keep_rms, ensemble, ensemble_stat)
        else:
            mix_shape = mix.shape
            if ensemble is not None:
                mix = mix.repeat(ensemble, 1, 1)
            mix = mix.to(torch.float32).contiguous()
            eng = self._get_engine()
            B, _, T = mix.shape
            # mean / median / signal_median reduce on the device inside the plan
            ens_mode = {"mean": 0, "median": 1, "signal_median": 2}[ensemble_stat] if ensemble is not None else None
            key = (B, T, int(n_steps), float(epsilon), bool(keep_rms), bool(use_aux_signal),
                   warm_start, ensemble, ens_mode)
            def make_plan(arena):
                return EnhancePlan(self._get_engine(), B, T, int(n_steps), float(epsilon), keep_rms=bool(keep_rms),
                                   use_aux_signal=bool(use_aux_signal), warm_start=warm_start,
                                   diff=dict(self.diff_kwargs), ensemble=ensemble,
                                   ensemble_mode=ens_mode, arena=arena)

            plan = self._arena_plan(key, 0, make_plan)
            try:
                x = plan(mix, rng, clone=True)[:, None, :]
            except L.OuRangeError as e:
                # a split-f16 operand left its range: widen the exponents of
                # the layers it names and rerun on the same noise
                nz = plan.NZ.clone()

                def rerun():
                    p = self._arena_plan(key, 0, make_plan)
                    return p.run_with_noise(mix, nz).clone()[:, None, :]

                x = self._range_recover(e, rerun)
        if x_ndim == 1:
            x = x[0, 0]
        elif x_ndim == 2:
            x = x[:, 0, :]
        return x

    def enhance_many(self, mixes, n_steps: Optional[int] = None, epsilon: Optional[float] = None,
                     rng: Optional[torch.Generator] = None, keep_rms: Optional[bool] = False, streams: int = 2,
                     pre_noise=None):
        """Enhance a sequence of clips (each a (T,), (B, T) or (B, 1, T) device
        tensor, as ``enhance`` takes them) with up to ``streams`` enhances in
        flight at once, on their own HIP streams and plans.  At batch 1 one
        enhance leaves most of the chip idle while its GRUs run (a serial
        801-step chain per clip); a second clip's convolutions fill it.  Each
        clip's result equals ``enhance`` of that clip with the noise drawn in
        clip order from ``rng``; ``pre_noise(i)``, if given, runs right before
        clip i draws its noise (the CLI discards other ranks' draws there).
        Returns the list of outputs."""
        from ...plan import EnhancePlan
        from ... import engine as E

        if epsilon is None:
            epsilon = self.diff_kwargs.epsilon
        if n_steps is None:
            n_steps = self.diff_kwargs.n_steps
        mixes = list(mixes)
        if not mixes:
            return []
        S = max(1, min(int(streams), E.MAX_SLOTS))
        eng = self._get_engine()
        streams_dev = getattr(self, "_streams_dev", None)
        if not hasattr(self, "_streams") or len(self._streams) < S or streams_dev != eng.device:
            self._streams = [torch.cuda.Stream(device=eng.device) for _ in range(S)]
            self._streams_dev = eng.device
        main = torch.cuda.current_stream(eng.device)
        shapes, outs, pending = [], [], []
        for i, mix in enumerate(mixes):
            nd = mix.ndim
            m3 = mix[None, None, :] if nd == 1 else mix[:, None, :] if nd == 2 else mix
            if nd > 3:
                raise ValueError("The input should have at most 3 dimensions")
            m3 = m3.to(torch.float32).contiguous()
            B, _, T = m3.shape
            slot = i % S
            # queued plans keep the conditioner's st_convs on its own lane: a
            # main lane that waits on the side lane early serialises two
            # clips in flight (865 -> 636 audio-s/s measured)
            key = (B, T, int(n_steps), float(epsilon), bool(keep_rms), False, None, None, None, slot, "queued")
            plan = self._arena_plan(key, slot, lambda ar: EnhancePlan(eng, B, T, int(n_steps), float(epsilon),
                                                                      keep_rms=bool(keep_rms),
                                                                      diff=dict(self.diff_kwargs), slot=slot,
                                                                      arena=ar, st_lane=False))
            self._inflight.add(key)
            if pre_noise is not None:
                pre_noise(i)
            st = self._streams[slot]
            st.wait_stream(main)   # the input was produced on the caller's stream
            with torch.cuda.stream(st):
                out = plan.submit(m3, rng).clone()
                nz = plan.NZ.clone()   # kept for a rerun with f32 operands
            out.record_stream(main)
            nz.record_stream(main)
            outs.append(out)
            shapes.append(nd)
            pending.append((key, m3, nz))
        for st in self._streams[:S]:
            main.wait_stream(st)
        try:
            try:
                plan.check()   # synchronises; the status word is shared by the engine's plans
            finally:
                self._inflight.clear()
        except L.OuRangeError as e:
            # as enhance(): widen the named layers' exponents (or fall back to
            # f32 operands) and rerun every clip of the call on its noise
            def rerun():
                eng = self._get_engine()
                res = []
                for key, m3, nz in pending:
                    B, _, T = m3.shape
                    p0 = self._arena_plan(key[:-2] + (0,), 0,
                                          lambda ar: EnhancePlan(eng, B, T, int(n_steps), float(epsilon),
                                                                 keep_rms=bool(keep_rms), diff=dict(self.diff_kwargs),
                                                                 arena=ar))
                    res.append(p0.run_with_noise(m3, nz).clone())
                return res

            outs = self._range_recover(e, rerun)
        res = []
        for x, nd in zip(outs, shapes):
            res.append(x[0] if nd == 1 else x if nd == 2 else x[:, None, :])
        return res

    def _range_recover(self, err, rerun, rounds=4):
        """Recover from a split-f16 range error: widen the staging exponents
        of the layers ``err`` names (Engine.widen_ranges: only those layers,
        the rest keep 2^-6) and ``rerun()`` -- the same noise, plans recorded
        again -- until a replay is clean.  An error that names no layer, an
        exponent past its limit, or ``rounds`` failed reruns switch the model
        to f32 operands instead (one counted fallback)."""
        log = os.environ.get("OUHIP_RANGE_LOG") == "1"   # diagnostics: each round's per-layer codes
        for _ in range(rounds):
            eng = self._engine
            if log:
                import sys

                print(f"[ou range] round {self.range_widenings + 1}: "
                      + " ".join(f"{type(eng.range_owners[s]).__name__}#{s}:{c:#x}" for s, c in err.flags),
                      file=sys.stderr, flush=True)
            if (eng is None or not getattr(err, "flags", ())
                    or not eng.widen_ranges(err.flags, consumers=getattr(err, "consumers", None))):
                break
            self.range_widenings += 1
            self._plans = collections.OrderedDict()   # exponents are read at record time
            try:
                return rerun()
            except L.OuRangeError as e2:
                err = e2
        self._conv_prec = 0
        self.range_fallbacks += 1
        self.invalidate()
        return rerun()

    @staticmethod
    def _ensemble_reduce(x, stat):
        """universe.py:359-368 for the known-answer mode (x: (E, B, 1, T) on
        the device): the same ou_ensemble_reduce / ou_signal_median kernels
        the recorded plans use."""
        from ...utils.stats import ensemble_reduce

        return ensemble_reduce(x, stat)

    def _enhance_fake_score(self, mix, n_steps, epsilon, target, fake_score_snr, rng, keep_rms,
                            ensemble, ensemble_stat):
        """The reference's built-in sampler known-answer mode
        (universe.py:278-298): the network is replaced by the true score plus
        noise at ``fake_score_snr`` dB.  It exercises only the sampler, so it
        runs as device tensor ops (no network is evaluated)."""
        from ...plan import sigma_schedule

        dev = mix.device
        mix_rms = mix.square().mean(dim=(-2, -1), keepdim=True).sqrt()
        if ensemble is not None:
            mix_shape = mix.shape
            mix = torch.stack([mix] * ensemble, dim=0).view((-1,) + mix_shape[1:])
        mix_len = mix.shape[-1]
        pad = self.tot_ds - mix_len % self.tot_ds
        mix = torch.nn.functional.pad(mix, (pad // 2, pad - pad // 2))
        target = torch.nn.functional.pad(target, (pad // 2, pad - pad // 2))
        from ...utils.norm import normalize_batch

        (mix, target), *_ = normalize_batch((mix, target), norm=2, **self.normalization_kwargs)
        snr = 5.0 if fake_score_snr is None else fake_score_snr

        def randn(shape):
            if rng is not None and rng.device != dev:
                return torch.randn(shape, generator=rng, device=rng.device).to(dev)
            return torch.randn(shape, generator=rng, device=dev)

        def score_fn(x, s):
            ts = -(x - target) / s[:, None, None] ** 2
            rms = (ts**2).mean().sqrt()
            return ts + randn(ts.shape) * (rms * 10 ** (-snr / 20.0))

        d = self.diff_kwargs
        delta_t = 1.0 / (n_steps - 1)
        gamma = (d.sigma_max / d.sigma_min) ** -delta_t
        eta = 1 - gamma**epsilon
        beta = math.sqrt(1 - gamma ** (2 * (epsilon - 1.0)))
        sigma = torch.from_numpy(sigma_schedule(d, n_steps)).to(dev)
        sigma = torch.broadcast_to(sigma[None, :], (mix.shape[0], n_steps))
        x = randn(mix.shape) * sigma[:, 0][:, None, None]
        for n in range(n_steps - 1):
            s_now, s_next = sigma[:, n], sigma[:, n + 1]
            score = score_fn(x, s_now)
            z = randn(x.shape) * s_next[:, None, None]
            x = x + s_now[..., None, None] ** 2 * eta * score + beta * z
        score = score_fn(x, sigma[:, -1])
        x = x + sigma[:, -1, None, None] ** 2 * score
        x = x[..., pad // 2: -(pad - pad // 2)]
        if keep_rms:
            x_rms = x.square().mean(dim=(-2, -1), keepdim=True).sqrt().clamp(min=1e-5)
            x = x * (mix_rms / x_rms)
        scale = abs(x).max(dim=-1, keepdim=True).values
        x = torch.where(scale > 1.0, x / scale, x)
        if ensemble is not None:
            x = self._ensemble_reduce(x.view((-1,) + tuple(mix_shape)), ensemble_stat)
        return x


class UniverseGAN(Universe):
    """UNIVERSE++ (universe_gan.py:62-151): Universe + the signal-decoupling
    layer used by ``use_aux_signal`` / ``warm_start``.  The discriminators are
    training losses and are not built (their checkpoint keys are skipped by
    the loader)."""

    def __init__(self, fs, normalization_norm, score_model, condition_model, diffusion,
                 losses=None, training=None, validation=None, optimizer=None, scheduler=None,
                 grad_clipper=None, transform=None, normalization_kwargs=None,
                 detach_cond=False, edm=None):
        super().__init__(fs, normalization_norm, score_model, condition_model, diffusion,
                         losses, training, validation, optimizer, scheduler, grad_clipper,
                         transform=None, normalization_kwargs=normalization_kwargs,
                         detach_cond=detach_cond, edm=edm)

    def init_losses(self, score_model, condition_model, losses, training):
        losses = losses or {}
        if losses.get("use_signal_decoupling", False):
            act = losses.get("signal_decoupling_act", None)
            if act != "snake":
                raise NotImplementedError("signal_decoupling_act must be 'snake'")
            self.signal_decoupling_layer = PReLU_Conv(self.n_channels, 1, 3, padding="same",
                                                      act_type="snake")
        else:
            self.signal_decoupling_layer = None

    def model_parameters(self):
        params = itertools.chain(self.get_score_model().parameters(), self.condition_model.parameters())
        if self.signal_decoupling_layer is not None:
            params = itertools.chain(params, self.signal_decoupling_layer.parameters())
        return params
