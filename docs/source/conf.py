# Sphinx configuration for the apex (MI355X) API docs.
#
# autodoc imports the package from the repository root; the compiled extension (apex._C) is
# mocked so the docs build on a machine without ROCm. Every module page is checked for
# importable targets by tests/test_docs.py (which runs without sphinx).
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

project = "apex (MI355X)"
author = "apex MI355X contributors"
copyright = "2026, apex MI355X contributors"
version = release = "0.2"

extensions = [
    "sphinx.ext.autodoc",
    "sphinx.ext.autosummary",
    "sphinx.ext.napoleon",
    "sphinx.ext.viewcode",
    "sphinx.ext.mathjax",
]
autodoc_mock_imports = ["apex._C"]
autodoc_member_order = "bysource"
autodoc_default_options = {"members": True, "undoc-members": False, "show-inheritance": True}
napoleon_google_docstring = True
napoleon_numpy_docstring = True

templates_path = []
source_suffix = ".rst"
master_doc = "index"
exclude_patterns = ["build"]
pygments_style = "sphinx"
html_theme = os.environ.get("APEX_DOCS_THEME", "alabaster")
html_static_path = ["_static"]
htmlhelp_basename = "apexdoc"
