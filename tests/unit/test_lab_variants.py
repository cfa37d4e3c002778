"""The A/B variant builds (tools/lab/build_variant.py) patch a copy of csrc/kernels by exact text
replacement: every pattern must still be present in the production sources, or a variant build
would fail (or, worse, silently measure the production kernel)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_variant_patterns_match_the_sources():
    spec = importlib.util.spec_from_file_location("build_variant", os.path.join(ROOT, "tools", "lab", "build_variant.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.VARIANTS
    for name, patches in mod.VARIANTS.items():
        for fname, old, new in patches:
            text = open(os.path.join(ROOT, "csrc", "kernels", fname)).read()
            assert text.count(old) >= 1, (name, fname, old)
            assert old != new, name
