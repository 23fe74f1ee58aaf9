"""Plotly figures of decision / objective space histories (reference ``vis_tools/plot.py``).

Same entry points and figure semantics as the reference: animated scatter of the
population per generation with a generation slider and play/pause buttons
(``plot_dec_space``, ``plot_obj_space_2d``, ``plot_obj_space_3d``), min/max/median/
mean fitness curves for single-objective runs (``plot_obj_space_1d``), optional
true Pareto front overlay and sorted-line drawing of 2-D fronts.  Inputs may be
lists of torch tensors (device tensors are moved to the host) or arrays.
"""
from __future__ import annotations

import numpy as np


def _np(x):
    try:
        import torch

        if isinstance(x, torch.Tensor):
            return x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(x)


def _go():
    try:
        import plotly.graph_objects as go
    except ImportError:  # pragma: no cover
        raise ImportError("The plot function requires plotly to be installed.")
    return go


def _range(arrs, col):
    allv = np.concatenate([a[:, col] for a in arrs])
    lo, hi = float(np.nanmin(allv)), float(np.nanmax(allv))
    span = hi - lo if hi > lo else 1.0
    return [lo - 0.1 * span, hi + 0.1 * span]


def _animated(frames_data, layout_extra, pf_trace=None, **kwargs):
    go = _go()
    frames, steps = [], []
    for i, data in enumerate(frames_data):
        d = list(data) + ([pf_trace] if pf_trace is not None else [])
        frames.append(go.Frame(data=d, name=str(i)))
        steps.append({"label": i, "method": "animate",
                      "args": [[str(i)], {"frame": {"duration": 200, "redraw": False}, "mode": "immediate", "transition": {"duration": 200}}]})
    sliders = [{"currentvalue": {"prefix": "Generation: "}, "pad": {"b": 1, "t": 10}, "len": 0.8, "x": 0.2, "y": 0,
                "yanchor": "top", "xanchor": "left", "steps": steps}]
    buttons = [{"args": [None, {"frame": {"duration": 200, "redraw": False}, "fromcurrent": True,
                                "transition": {"duration": 200, "easing": "linear"}, "mode": "immediate"}],
                "label": "Play", "method": "animate"},
               {"args": [[None], {"frame": {"duration": 0, "redraw": False}, "mode": "immediate", "transition": {"duration": 0}}],
                "label": "Pause", "method": "animate"}]
    layout = go.Layout(legend={"x": 1, "y": 1, "xanchor": "auto"}, margin={"l": 0, "r": 0, "t": 0, "b": 0}, sliders=sliders,
                       updatemenus=[{"type": "buttons", "buttons": buttons, "x": 0.2, "xanchor": "right", "y": 0, "yanchor": "top",
                                     "direction": "left", "pad": {"r": 10, "t": 30}}], **layout_extra, **kwargs)
    return go.Figure(data=frames[0].data, layout=layout, frames=frames)


def plot_dec_space(population_history, **kwargs):
    go = _go()
    pops = [_np(p) for p in population_history]
    data = [[go.Scatter(x=p[:, 0], y=p[:, 1], mode="markers", marker={"color": "#636EFA"})] for p in pops]
    return _animated(data, {"xaxis": {"range": _range(pops, 0)}, "yaxis": {"range": _range(pops, 1)}}, **kwargs)


def plot_obj_space_1d(fitness_history, animation=True, **kwargs):
    return plot_obj_space_1d_animation(fitness_history, **kwargs) if animation else plot_obj_space_1d_no_animation(fitness_history, **kwargs)


def _stats(fitness_history):
    fh = [_np(f).reshape(-1) for f in fitness_history]
    return (np.arange(len(fh)), [float(np.min(f)) for f in fh], [float(np.max(f)) for f in fh],
            [float(np.median(f)) for f in fh], [float(np.mean(f)) for f in fh])


def plot_obj_space_1d_no_animation(fitness_history, **kwargs):
    go = _go()
    g, mn, mx, md, av = _stats(fitness_history)
    return go.Figure([go.Scatter(x=g, y=v, mode="lines", name=n) for v, n in ((mn, "Min"), (mx, "Max"), (md, "Median"), (av, "Average"))],
                     layout=go.Layout(legend={"x": 1, "y": 1, "xanchor": "auto"}, margin={"l": 0, "r": 0, "t": 0, "b": 0}, **kwargs))


def plot_obj_space_1d_animation(fitness_history, **kwargs):
    go = _go()
    g, mn, mx, md, av = _stats(fitness_history)
    data = [[go.Scatter(x=g[: i + 1], y=v[: i + 1], mode="lines", name=n) for v, n in ((mn, "Min"), (mx, "Max"), (md, "Median"), (av, "Average"))]
            for i in range(len(g))]
    lo, hi = min(mn), max(mx)
    span = hi - lo if hi > lo else 1.0
    return _animated(data, {"xaxis": {"range": [0, len(g)]}, "yaxis": {"range": [lo - 0.1 * span, hi + 0.1 * span]}}, **kwargs)


def plot_obj_space_2d(fitness_history, problem_pf=None, sort_points=False, **kwargs):
    go = _go()
    fh = [_np(f) for f in fitness_history]
    pf = None
    if problem_pf is not None:
        p = _np(problem_pf)
        p = p[np.argsort(p[:, 0])]
        pf = go.Scatter(x=p[:, 0], y=p[:, 1], mode="lines" if sort_points else "markers", name="Pareto Front",
                        marker={"color": "#FFA15A", "size": 2})
    data = []
    for f in fh:
        if sort_points:
            f = f[np.argsort(f[:, 0])]
        data.append([go.Scatter(x=f[:, 0], y=f[:, 1], mode="lines+markers" if sort_points else "markers", name="Population",
                                marker={"color": "#636EFA"})])
    return _animated(data, {"xaxis": {"range": _range(fh, 0)}, "yaxis": {"range": _range(fh, 1)}}, pf_trace=pf, **kwargs)


def plot_obj_space_3d(fitness_history, sort_points=False, problem_pf=None, **kwargs):
    go = _go()
    fh = [_np(f) for f in fitness_history]
    pf = None
    if problem_pf is not None:
        p = _np(problem_pf)
        pf = go.Scatter3d(x=p[:, 0], y=p[:, 1], z=p[:, 2], mode="markers", name="Pareto Front", marker={"color": "#FFA15A", "size": 2})
    data = [[go.Scatter3d(x=f[:, 0], y=f[:, 1], z=f[:, 2], mode="markers", name="Population", marker={"color": "#636EFA", "size": 3})]
            for f in fh]
    scene = {"xaxis": {"range": _range(fh, 0)}, "yaxis": {"range": _range(fh, 1)}, "zaxis": {"range": _range(fh, 2)}, "aspectmode": "cube"}
    return _animated(data, {"scene": scene}, pf_trace=pf, **kwargs)
