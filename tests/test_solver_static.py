"""CPU: static properties of the solver's GPU orchestration (solver.py), checked on its source.

Every HIP-graph capture must use the thread-local capture mode: with an RCCL process group
alive its watchdog thread queries events, and under the default global mode such a query
invalidates an ongoing capture (found by the round-3 RCCL test).
"""
import ast
import inspect

from deeppde_actorcritic_amd import solver as psol


def _graph_calls():
    tree = ast.parse(inspect.getsource(psol))
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr == "graph":
            yield node


def test_every_graph_capture_is_thread_local():
    assert psol._CAPTURE_MODE == "thread_local"
    calls = list(_graph_calls())
    assert len(calls) >= 6  # _GradGraph, _SplitActorGraphs (2), _SplitCriticGraphs (3)
    for c in calls:
        kw = {k.arg: k.value for k in c.keywords}
        assert "capture_error_mode" in kw, ast.dump(c)
        v = kw["capture_error_mode"]
        assert isinstance(v, ast.Name) and v.id == "_CAPTURE_MODE", ast.dump(v)


def test_gback_default_and_choices():
    assert psol.GBACK in ("early", "late")
