"""Launch plans: one recorded ``ou_program`` per (shape, options).

* :class:`EnhancePlan`   -- Universe.enhance (universe.py:231-375), whole sampler
* :class:`ScorePlan`     -- ScoreNetwork.forward (score.py:278-298)
* :class:`CondPlan`      -- ConditionerNetwork.forward (condition.py:346-377)

Buffers are allocated once per plan (caller-owned device memory from the torch
allocator); the recorded program holds raw pointers into them, so a plan can be
replayed as a single hipGraph.  All arithmetic on the sampler's scalars
(sigma schedule, EDM weights, update coefficients) is done here once, in
float32 exactly as the reference's tensor ops round them.
"""
import math
import os

import numpy as np
import torch

from . import _lib as L
from . import engine as E
from .engine import Act, new_act

f32 = np.float32


def sigma_schedule(diff, n_steps):
    """get_std_dev over the reversed linspace (universe.py:307-311,380-386),
    evaluated with float32 tensor ops like the reference."""
    if diff.get("schedule", "geometric") != "geometric":
        raise NotImplementedError()
    time = torch.linspace(0, 1, n_steps, dtype=torch.float32).flip(dims=[0])
    s_min, s_max = diff["sigma_min"], diff["sigma_max"]
    return (s_min * (s_max / s_min) ** time).numpy().astype(np.float32)


def edm_weights(s, level_db, data_level_db=None):
    """_get_edm_weights (universe.py:175-189) for a float32 sigma."""
    lvl = level_db if data_level_db is None else data_level_db
    sd = 10.0 ** (lvl / 20.0)
    s = f32(s)
    s2 = f32(s * s)
    den = f32(s2 + f32(sd**2))
    sn = f32(np.sqrt(den))
    return {
        "skip": f32(f32(sd**2) / den),
        "in": f32(f32(1.0) / sn),
        "out": f32(f32(s * f32(sd)) / sn),
    }


# EnhancePlan.__call__ reads the status words through pinned memory after one
# stream wait, the result copy queued before it (+0.6 % over a blocking read,
# profiles/ab_r04_summary.txt)
PINNED_CHECK = True

# OUHIP_NOISE_GRAPH=0: draw the sampler's noise with one torch.randn call per
# draw instead of replaying them as one captured graph
NOISE_GRAPH = os.environ.get("OUHIP_NOISE_GRAPH", "1") != "0"


class NoiseDraws:
    """The sampler's n device-generator draws ``torch.randn(shape, generator=rng,
    out=nz[k])``, k = 0..n-1 (universe.py:39-41,326,338), replayed as one
    captured graph per generator: the graph-safe Philox path reads the
    generator's seed / offset at replay and advances it by the draws' total,
    so the values and the generator's state afterwards are those of the n
    eager calls -- checked once per generator against eager draws from a copy
    of its state (a mismatch, or a capture error, falls back to the eager
    calls for that generator).  One launch instead of n: the draws sit between
    two enhances, where the GPU idles while the host issues them."""

    def __init__(self, nz, shape):
        self.nz, self.shape = nz, shape
        self.graphs = {}   # id(generator) -> (generator, graph; False: seen once; None: eager)

    def _eager(self, rng, out):
        for k in range(out.shape[0]):
            torch.randn(self.shape, generator=rng, out=out[k])

    def _capture(self, rng):
        gen = rng if rng is not None else torch.cuda.default_generators[self.nz.device.index or 0]
        state = gen.get_state()
        try:
            g = torch.cuda.CUDAGraph()
            if rng is not None:
                g.register_generator_state(rng)
            with torch.cuda.graph(g):
                self._eager(rng, self.nz)
            # the check: one replay against eager draws from a copy of the state
            chk = torch.Generator(device=self.nz.device)
            chk.set_state(state)
            ref = torch.empty_like(self.nz)
            self._eager(chk, ref)
            g.replay()
            ok = bool(torch.equal(ref, self.nz)) and bool(torch.equal(chk.get_state(), gen.get_state()))
        except Exception:   # noqa: BLE001 -- any capture trouble: the eager draws
            g, ok = None, False
        gen.set_state(state)   # the check consumed nothing of the caller's stream
        return g if ok else None

    def draw(self, rng):
        """A generator's first draw is eager; its second captures the graph (a
        generator used once never pays for a capture)."""
        if not NOISE_GRAPH or self.nz.shape[0] < 2:
            self._eager(rng, self.nz)
            return
        ent = self.graphs.get(id(rng))
        if ent is None or ent[0] is not rng:   # first sight
            if len(self.graphs) >= 4:
                self.graphs.clear()
            self.graphs[id(rng)] = (rng, False)
            self._eager(rng, self.nz)
            return
        if ent[1] is False:   # second sight: capture (None: capture failed or mismatched)
            ent = self.graphs[id(rng)] = (rng, self._capture(rng))
        if ent[1] is None:
            self._eager(rng, self.nz)
        else:
            ent[1].replay()


class _PlanBase:
    def __init__(self, eng):
        self.eng = eng
        self.dev = eng.device
        self.prog = L.Program()
        E.begin_record(eng.conv_prec, eng.device)

    def __init_subclass__(cls, **kw):
        # every subclass records in its __init__: close the recording context
        # when it returns (or raises)
        super().__init_subclass__(**kw)
        init = cls.__init__

        def wrapped(self, *a, **k):
            try:
                init(self, *a, **k)
            finally:
                E.end_record()
                E._GRU_WS_ZEROED = False
                E._LANE = 0
                E._SLOT = 0
                E._ARENA = None

        cls.__init__ = wrapped

    def _launch(self, stream, use_graph):
        # A plan's first replay is eager (native launch loop) and the hipGraph is
        # captured from its second replay on, so a plan used once (a clip of a
        # new length) does not pay for graph instantiation (OUHIP_EAGER_FIRST=0
        # captures at once).  The programs' capture and side-lane streams are
        # process-wide (csrc/ou_program.hip): per-program streams had bound two
        # callers' streams to one hardware queue and serialised them.
        self.uses = getattr(self, "uses", 0) + 1
        import os

        eager_first = os.environ.get("OUHIP_EAGER_FIRST", "1") != "0"
        use_graph = use_graph and os.environ.get("OUHIP_GRAPH", "1") != "0"   # 0: always the native launch loop
        if use_graph and (self.uses > 1 or self.prog.captured or not eager_first):
            if not self.prog.captured:
                self.prog.capture()
            self.prog.launch(stream)
        else:
            self.prog.run(stream)

    def check(self, pinned=False):
        """Raise on a GRU hand-off timeout (status word 0) or a split-f16
        range error: OuRangeError.flags lists the (layer slot, range code)
        pairs of the engine's per-layer words (Engine.widen_ranges)."""
        n = 4 + len(self.eng.range_owners)
        st = self.eng.status[:n]
        if pinned:
            # one wait: the status words ride to pinned host memory on the
            # stream behind the replay, instead of a blocking read issued
            # after it (a second host wake-up per call)
            hs = getattr(self.eng, "status_host", None)
            if hs is None or hs.numel() != n:
                hs = self.eng.status_host = torch.empty(st.shape, dtype=st.dtype, pin_memory=True)
            hs.copy_(st, non_blocking=True)
            torch.cuda.current_stream(self.dev).synchronize()
            flags = hs.tolist()
        else:
            flags = st.tolist()
        if any(flags):
            st.zero_()
            if flags[0]:
                raise L.OuHipError("GRU recurrence timed out (workgroup hand-off never completed)")
            per_layer = [(i - 4, f) for i, f in enumerate(flags) if i >= 4 and f]
            e = L.OuRangeError("split-f16 operand out of range (range codes %s%s)"
                               % (per_layer[:8], ", shared word %d" % flags[1] if flags[1] else ""))
            e.flags = per_layer if not flags[1] else []   # a shared-word flag names no layer
            e.consumers = dict(self.prog.__dict__.get("split_consumers", {}))   # this plan's split-image pairs
            raise e


class EnhancePlan(_PlanBase):
    """The whole enhance() for a fixed (batch, length, n_steps, options)."""

    def __init__(self, eng, batch, mix_len, n_steps, epsilon, keep_rms=False,
                 use_aux_signal=False, warm_start=None, diff=None, ensemble=None,
                 ensemble_mode=None, slot=0, arena=None, st_lane=True):
        # arena: record every buffer into this Arena (engine.Arena; the caller
        # owns it and retries with a bigger one on ArenaFull)
        if arena is not None:
            arena.off = 0
            E._ARENA = arena
        self.arena = arena
        super().__init__(eng)
        # plans that may run concurrently (Universe.enhance_many) use their own
        # K-slice workspaces: engine.conv_desc offsets by the recording slot
        assert 0 <= slot < E.MAX_SLOTS
        E._SLOT = slot
        dev, B = self.dev, batch
        self.B, self.mix_len, self.n_steps = B, mix_len, n_steps
        tot = eng.tot_ds
        self.pad = tot - mix_len % tot
        Tp = mix_len + self.pad
        self.Tp = Tp
        self.use_aux = use_aux_signal
        self.warm = warm_start
        diff = diff or eng.cfg["diffusion"]
        # sampler constants (universe.py:301-305)
        delta_t = 1.0 / (n_steps - 1)
        gamma = (diff["sigma_max"] / diff["sigma_min"]) ** -delta_t
        eta = 1 - gamma**epsilon
        beta = math.sqrt(1 - gamma ** (2 * (epsilon - 1.0)))
        sig = sigma_schedule(diff, n_steps)
        self.sigma = sig
        edm = eng.edm
        n_start = 0 if warm_start is None else int(warm_start)
        self.n_start = n_start
        # buffers
        self.MIX = E.empty((B, 1, mix_len), dtype=torch.float32, device=dev)
        self.XP = new_act(B, 1, Tp, dev)
        self.XN = new_act(B, 1, Tp, dev)
        self.X = new_act(B, 1, Tp, dev)
        n_noise = 0 if use_aux_signal else 1 + (n_steps - 1 - n_start)
        self.n_noise = n_noise
        self.NZ = E.empty((max(n_noise, 1), B, 1, Tp), dtype=torch.float32, device=dev)
        self.OUT = E.empty((B, mix_len), dtype=torch.float32, device=dev)
        self.MIXRMS = E.empty((B,), dtype=torch.float32, device=dev)
        cb = eng.alloc_cond(B, Tp, need_aux=use_aux_signal or warm_start is not None)
        self.cb = cb
        p = self.prog
        # the GRU hand-off workspaces are zeroed once per replay; the GRU
        # launches then skip their per-launch memsets (ou_gru_desc.ws_zeroed)
        E.rec_gru_ws_zero(p, cb["gran"])
        E._GRU_WS_ZEROED = True
        # ---- record ----
        mixact = Act(self.MIX)
        p.label = "prep"
        if keep_rms:
            p.add(L.OP_RMS, L.RmsArgs(x=mixact.ptr, out=self.MIXRMS.data_ptr(), batch=B,
                                      n=mix_len, denom=float(mix_len), eps=0.0))
        p.add(L.OP_PAD, L.PadArgs(x=mixact.ptr, x_bstride=mix_len, y=self.XP.ptr, batch=B,
                                  n_in=mix_len, n_out=Tp, left=self.pad // 2))
        level = 10 ** (eng.level_db / 20.0)
        p.add(L.OP_NORMALIZE, L.NormArgs(x=self.XP.ptr, y=self.XN.ptr, batch=B, n=Tp,
                                         level=level, eps=1e-5))
        # The conditioner (and the loop-invariant signal_cond_proj convs) run
        # on lane 1 concurrently with lane 0's first score-network encoder and
        # bottleneck GRU, which do not read the conditions (score.py:284-286);
        # lane 0 waits for them right before the first decoder.  Not with the
        # aux / warm-start paths, whose initial sample needs the conditioner.
        self.overlap = E.overlap_enabled() and not use_aux_signal and warm_start is None
        ev_cond = {}
        after_level = None
        if self.overlap:
            # condition l is projected (signal_cond_proj) and signalled as soon
            # as the conditioner's decoder level l has produced it: the score
            # decoder of the first pass waits level by level
            ev_in = p.signal()
            E.set_lane(p, 1)
            p.wait(ev_in)
            self.SC = eng.alloc_sc(B, Tp)

            # the projections run on their own lane (E.SC_LANE), so the
            # conditioner's next decoder level does not queue behind them --
            # not in enhance_many's plans (st_lane=False): the side-lane
            # streams are process-wide, and two plans in flight would
            # serialise on it
            sc_lane = st_lane

            def after_level(l, cond):
                if sc_lane:
                    ev = p.signal()
                    E.set_lane(p, E.SC_LANE)
                    p.wait(ev)
                p.label = f"cond sc{l}"
                p.add(L.OP_CONV, E.conv_desc(eng.s_sc[l], cond, self.SC[l]))
                ev_cond[l] = p.signal()
                if sc_lane:
                    E.set_lane(p, 1)
        conds, yaux = eng.rec_cond(p, cb, self.XN, need_aux=use_aux_signal or warm_start is not None,
                                   after_level=after_level, st_lane=0 if (self.overlap and st_lane) else None)
        if use_aux_signal or warm_start is not None:
            self.AUXT = new_act(B, yaux.C, Tp, dev)
            self.SIG = new_act(B, 1, Tp, dev)
            if eng.has_sdl:
                eng.rec_aux(p, yaux, self.AUXT, self.SIG.ptr, B, Tp)
            else:
                raise NotImplementedError("aux signal without a signal-decoupling layer")
        # lane 1's last signal (the sc lane took the conditions'): lane 0 joins it before finish
        ev_c1 = p.signal() if self.overlap and st_lane else None
        if use_aux_signal:
            x_final = self.SIG
        else:
            if self.overlap:
                E.set_lane(p, 0)
            else:
                self.SC = eng.alloc_sc(B, Tp)
                eng.rec_sc(p, conds, self.SC)
            # FiLM parameters for every step at once (noise embedding, K7)
            steps = list(range(n_start, n_steps))
            snet = np.array([(f32(edm["noise"]) * sig[n]) if edm is not None else sig[n]
                             for n in range(n_steps)], dtype=np.float32)
            self.SNET = torch.from_numpy(snet).to(dev)
            self.FILM = E.empty((n_steps, eng.film_rows), dtype=torch.float32, device=dev)
            self.GBUF = E.empty((n_steps, eng.emb_dim), dtype=torch.float32, device=dev)
            p.label = "score embed"
            eng.rec_embed(p, self.SNET, n_steps, self.FILM, self.GBUF)
            win = np.ones((n_steps, B), dtype=np.float32)
            coefs = []
            for n in range(n_steps):
                s_now = f32(sig[n])
                c = {"s2": f32(s_now * s_now)}
                if edm is not None:
                    w = edm_weights(s_now, eng.level_db, edm.get("data_level_db"))
                    win[n, :] = w["in"]
                    c.update(w_skip=w["skip"], w_out=w["out"])
                if n < n_steps - 1:
                    c.update(c_score=f32(f32(s_now * s_now) * f32(eta)), c_noise=f32(beta),
                             s_next=f32(sig[n + 1]))
                else:
                    c.update(c_score=f32(s_now * s_now))
                coefs.append(c)
            self.WIN = torch.from_numpy(win).to(dev)
            self.sb = eng.alloc_score(B, Tp)
            E.rec_gru_ws_zero(p, self.sb["gran"])   # lane 0, ahead of the first score GRU
            # initial sample (universe.py:322-331)
            if warm_start is None:
                p.add(L.OP_SCALE, L.ScaleArgs(z=self.NZ.data_ptr(), y=self.X.ptr, n=B * Tp,
                                              scale=float(sig[0]), add=0))
            else:
                p.add(L.OP_SCALE, L.ScaleArgs(z=self.NZ.data_ptr(), y=self.X.ptr, n=B * Tp,
                                              scale=float(sig[n_start]), add=self.SIG.ptr))
            film_base = self.FILM.data_ptr()
            zi = 1
            for n in steps:
                join = (lambda l: p.wait(ev_cond[l])) if (ev_cond and n == steps[0]) else None
                last = n == n_steps - 1
                film = film_base + 4 * n * eng.film_rows
                in_scale = self.WIN[n].data_ptr() if edm is not None else 0
                head = eng.head_desc(None, self.X.ptr, B, Tp, mode=2 if last else 1, x_ptr=self.X.ptr,
                                     z_ptr=0 if last else self.NZ[zi].data_ptr(), coef=coefs[n])
                eng.rec_score(p, self.sb, self.X, film, 0, in_scale=in_scale, sc_list=self.SC, before_level=join,
                              head=head)
                zi += 0 if last else 1
            x_final = self.X
        if ev_c1 is not None:
            p.wait(ev_c1)   # long done: the conditions were waited on in the first step
        p.label = "finish"
        p.add(L.OP_FINISH, L.FinishArgs(x=x_final.ptr, x_bstride=Tp, left=self.pad // 2,
                                        batch=B, len=mix_len, y=self.OUT.data_ptr(),
                                        mix_rms=self.MIXRMS.data_ptr() if keep_rms else 0))
        # ensemble reduction (universe.py:359-368): B = E x B0 results -> B0
        # (mode 0 mean, 1 median, 2 signal_median)
        self.RED = None
        if ensemble is not None and ensemble_mode is not None:
            assert B % ensemble == 0
            B0 = B // ensemble
            self.RED = E.empty((B0, mix_len), dtype=torch.float32, device=dev)
            # signal_median (mode 2): per-batch-item vote counts
            self.CNT = E.zeros((B0, 32), dtype=torch.int32, device=dev)
            p.add(L.OP_ENSEMBLE, L.EnsembleArgs(x=self.OUT.data_ptr(), y=self.RED.data_ptr(),
                                                ensemble=ensemble, mode=ensemble_mode,
                                                n=B0 * mix_len, batch=B0, counts=self.CNT.data_ptr()))

    def draw_noise(self, rng):
        """Noise in the reference's draw order (universe.py:39-41,326,338):
        x0 first, then one z per intermediate step."""
        shape = (self.B, 1, self.Tp)
        if rng is not None and rng.device != self.NZ.device:
            for k in range(self.n_noise):
                z = torch.randn(shape, generator=rng, device=rng.device, dtype=torch.float32)
                self.NZ[k].copy_(z, non_blocking=False)
            return
        nd = self.__dict__.get("_noise")
        if nd is None:
            nd = self._noise = NoiseDraws(self.NZ[: self.n_noise], shape)
        nd.draw(rng)

    def __call__(self, mix, rng=None, use_graph=True, clone=False):
        out = self.submit(mix, rng, use_graph)
        if clone and PINNED_CHECK:   # the copy of the result queued behind the replay, before the wait
            out = out.clone()
        self.check(pinned=PINNED_CHECK)
        return out.clone() if clone and not PINNED_CHECK else out

    def submit(self, mix, rng=None, use_graph=True):
        """Enqueue one enhance on the current stream without waiting for it
        (the caller checks the status word after synchronising)."""
        assert mix.shape == (self.B, 1, self.mix_len), mix.shape
        self.MIX.copy_(mix)
        self.draw_noise(rng)
        stream = torch.cuda.current_stream(self.dev).cuda_stream
        self._launch(stream, use_graph)
        return self.OUT if self.RED is None else self.RED

    def run_with_noise(self, mix, nz):
        """Rerun on noise drawn earlier (NZ of a plan of the same shape)."""
        self.MIX.copy_(mix)
        self.NZ.copy_(nz)
        self._launch(torch.cuda.current_stream(self.dev).cuda_stream, True)
        self.check()
        return self.OUT if self.RED is None else self.RED


class ScorePlan(_PlanBase):
    """ScoreNetwork.forward(x, sigma, cond) for a fixed (B, T)."""

    def __init__(self, eng, B, T):
        super().__init__(eng)
        dev = self.dev
        self.B, self.T = B, T
        self.XIN = new_act(B, 1, T, dev)
        self.SIG = torch.empty(B, dtype=torch.float32, device=dev)
        self.OUT = new_act(B, 1, T, dev)
        self.SC = eng.alloc_sc(B, T)
        self.CIN = [new_act(B, s.C, s.T, dev) for s in self.SC]
        self.FILM = torch.empty((B, eng.film_rows), dtype=torch.float32, device=dev)
        self.GBUF = torch.empty((B, eng.emb_dim), dtype=torch.float32, device=dev)
        self.sb = eng.alloc_score(B, T)
        p = self.prog
        eng.rec_embed(p, self.SIG, B, self.FILM, self.GBUF)
        eng.rec_sc(p, self.CIN, self.SC)
        eng.rec_score(p, self.sb, self.XIN, self.FILM.data_ptr(), eng.film_rows, sc_list=self.SC,
                      head=eng.head_desc(None, self.OUT.ptr, B, T, mode=0))

    def __call__(self, x, sigma, cond, use_graph=False):
        self.XIN.t.copy_(x)
        self.SIG.copy_(sigma.reshape(-1).to(torch.float32))
        for dst, src in zip(self.CIN, cond):
            dst.t.copy_(src)
        self._launch(torch.cuda.current_stream(self.dev).cuda_stream, use_graph)
        self.check()
        return self.OUT.t


class CondPlan(_PlanBase):
    """ConditionerNetwork.forward(x, train=True) for a fixed (B, T)."""

    def __init__(self, eng, B, T, need_aux=True):
        super().__init__(eng)
        self.B, self.T = B, T
        self.XIN = new_act(B, 1, T, self.dev)
        self.cb = eng.alloc_cond(B, T, need_aux=need_aux)
        self.conds, self.y = eng.rec_cond(self.prog, self.cb, self.XIN, need_aux=need_aux)

    def __call__(self, x, use_graph=False):
        self.XIN.t.copy_(x)
        self._launch(torch.cuda.current_stream(self.dev).cuda_stream, use_graph)
        self.check()
        return [c.t for c in self.conds], self.y.t, self.cb["H"].t
