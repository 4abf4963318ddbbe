"""INTEGRATION.md §2 overlay: with CGR_MPNN_3D_REFERENCE set, the reference checkout's own
sub-packages (data / training / utils) resolve to its files and ``models`` to ours.  Uses a stand-in
checkout tree (no reference code is imported or executed)."""

import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_overlay_resolves_reference_subpackages_and_our_models(tmp_path):
    ref = tmp_path / "checkout"
    for sub in ("data", "training", "utils", "models"):
        (ref / "cgr_mpnn_3D" / sub).mkdir(parents=True)
    (ref / "cgr_mpnn_3D" / "__init__.py").write_text("")
    (ref / "cgr_mpnn_3D" / "utils" / "__init__.py").write_text("")
    (ref / "cgr_mpnn_3D" / "utils" / "json_dumper.py").write_text("MARK = 'reference'\n")
    (ref / "cgr_mpnn_3D" / "training" / "trainer.py").write_text("MARK = 'trainer'\n")
    (ref / "cgr_mpnn_3D" / "models" / "GNN.py").write_text("raise ImportError('shadowed')\n")
    code = textwrap.dedent("""
        import importlib.util, cgr_mpnn_3D
        from cgr_mpnn_3D.utils import json_dumper
        from cgr_mpnn_3D.training import trainer
        spec = importlib.util.find_spec("cgr_mpnn_3D.models.GNN")
        print(json_dumper.MARK, trainer.MARK, spec.origin)
    """)
    env = dict(os.environ, CGR_MPNN_3D_REFERENCE=str(ref),
               PYTHONPATH=os.path.join(REPO, "cgr-mpnn-3d_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         check=True).stdout.split()
    assert out[:2] == ["reference", "trainer"]
    assert out[2].startswith(os.path.join(REPO, "cgr-mpnn-3d_amd"))
