"""The Sphinx API pages (docs/source/*.rst) only name things that exist: every automodule /
autoclass / autofunction target and every explicit ``:members:`` entry resolves to an importable
object, so the docs cannot silently rot (sphinx itself is not installed in the runtime image).
Every page is reachable from index.rst's toctrees."""
import importlib
import os
import re

import pytest

DOCS = os.path.join(os.path.dirname(__file__), "..", "docs", "source")
if not os.path.isdir(DOCS):  # e.g. a GPU-box snapshot that leaves the docs out (.gpurunignore)
    pytest.skip("docs/source not present", allow_module_level=True)
DIRECTIVE = re.compile(r"^\.\. (automodule|autoclass|autofunction|currentmodule):: (\S+)")


def _pages():
    return sorted(f for f in os.listdir(DOCS) if f.endswith(".rst"))


def _resolve(name):
    parts = name.split(".")
    for i in range(len(parts), 0, -1):
        try:
            obj = importlib.import_module(".".join(parts[:i]))
        except ImportError:
            continue
        for p in parts[i:]:
            obj = getattr(obj, p)
        return obj
    raise ImportError(name)


@pytest.mark.parametrize("page", _pages())
def test_autodoc_targets_resolve(page):
    current = None
    lines = open(os.path.join(DOCS, page)).read().splitlines()
    n = 0
    i = 0
    while i < len(lines):
        m = DIRECTIVE.match(lines[i])
        i += 1
        if not m:
            continue
        kind, target = m.groups()
        if kind in ("automodule", "currentmodule"):
            mod = importlib.import_module(target)
            current = target
            n += kind == "automodule"
            # explicit member lists may continue over indented lines
            opts = []
            while i < len(lines) and (lines[i].startswith("    ") or not lines[i].strip()):
                if not lines[i].strip():
                    break
                opts.append(lines[i].strip())
                i += 1
            text = " ".join(opts)
            mm = re.search(r":members:\s*(.*?)(?=\s:\w|$)", text)
            if kind == "automodule" and mm and mm.group(1).strip():
                for member in (s.strip() for s in mm.group(1).split(",")):
                    if member:
                        assert hasattr(mod, member), f"{page}: {target}.{member}"
                        n += 1
            continue
        full = target if "." in target and not current else f"{current}.{target}" if current else target
        _resolve(full)
        n += 1
    assert n > 0 or page == "index.rst", f"{page} documents nothing"


def test_every_page_in_a_toctree():
    index = open(os.path.join(DOCS, "index.rst")).read()
    listed = set(re.findall(r"^   (\w+)\s*$", index, re.M))
    for page in _pages():
        if page != "index.rst":
            assert page[:-4] in listed, page
