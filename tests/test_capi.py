"""C-ABI surface checks that need no GPU: the library loads and exports every
function include/avz.h declares; error strings; plan validation paths that run on
the host only."""
import ctypes as ct
import os
import re

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "avz.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(avz_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = declared()
    for n in ("avz_plan_create", "avz_plan_destroy", "avz_mvdr_batch", "avz_stft", "avz_strerror"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from avz import _lib
    for n in declared():
        assert hasattr(_lib.lib, n), n
    assert set(_lib.EXPORTED) <= set(declared())


def test_strerror_and_host_side_validation():
    from avz import _lib
    lib = _lib.lib
    assert lib.avz_strerror(0) == b"ok"
    assert lib.avz_strerror(-4) == b"unsupported configuration"
    assert lib.avz_version() == _lib.ABI_VERSION == 3
    assert b"aligned" in lib.avz_strerror(_lib.AVZ_ERR_ALIGN)
    c = _lib.AvzConfig(fs=16000, n_fft=768, hop=384, sigma=1.0, angle_deg=90.0, mic_d=0.01,
                       c_sound=343.0, fmin_hz=100.0, mask_mode=0, postfilter=1, pf_floor=0.05,
                       weight_eps=0.0, normalize=1, norm_eps=0.0, max_batch=1, max_samples=4096)
    h = ct.c_void_p()
    assert lib.avz_plan_create(ct.byref(h), ct.byref(c)) == _lib.AVZ_ERR_UNSUPPORTED
    c.n_fft, c.hop = 1024, 256
    assert lib.avz_plan_create(ct.byref(h), ct.byref(c)) == _lib.AVZ_ERR_UNSUPPORTED
    c.hop, c.mask_mode, c.postfilter = 512, 1, 1    # IBM post-filter needs the IBM mask
    assert lib.avz_plan_create(ct.byref(h), ct.byref(c)) == _lib.AVZ_ERR_ARG
    c.postfilter, c.max_samples = 0, 100            # shorter than one frame
    assert lib.avz_plan_create(ct.byref(h), ct.byref(c)) == _lib.AVZ_ERR_ARG
    assert lib.avz_mvdr_batch(None, None, None) == _lib.AVZ_ERR_ARG
    # scene generator: source Philox streams must stay below the noise streams (0x100 + mic),
    # and the 0.25-s envelope block must be non-empty; rejected before any device work
    gen = lambda k, fs: lib.avz_scene_generate(1, 0, k, 16000, 0, 0.01, 343.0, fs, 0.0,  # noqa
                                               30.0, None, 0, 0, None, None, 0, None, 0, None)
    assert gen(256, 16000.0) == _lib.AVZ_ERR_ARG  # sources 0..255 keep their Philox streams distinct
    assert gen(2, 3.0) == _lib.AVZ_ERR_ARG
    assert gen(2, float("nan")) == _lib.AVZ_ERR_ARG


def test_ctypes_struct_layout_matches_header(tmp_path):
    """Compile a probe against include/avz.h with gcc and compare every field offset."""
    import subprocess
    from avz import _lib
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', 'int main(void){']
    for cname, cls in (("avz_config", _lib.AvzConfig), ("avz_batch_args", _lib.AvzBatchArgs)):
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    for cname, cls in (("avz_config", _lib.AvzConfig), ("avz_batch_args", _lib.AvzBatchArgs)):
        assert int(got[cname]) == ct.sizeof(cls)
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_integration_shim_structs_match_the_host_layer():
    """The reference-side ctypes shim printed in INTEGRATION.md declares the same struct
    fields (names and C types, in order) as avz._lib, which the header-layout test above
    pins to include/avz.h: a stale shim would hand the library a short struct."""
    import ast
    import textwrap
    from avz import _lib
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, re.S)
    shim = {}
    for b in blocks:
        for node in ast.walk(ast.parse(textwrap.dedent(b))):
            if isinstance(node, ast.ClassDef):
                for st in node.body:
                    if isinstance(st, ast.Assign) and st.targets[0].id == "_fields_":
                        shim[node.name] = eval(compile(ast.Expression(st.value), "shim", "eval"),
                                               {"ct": ct})
    assert {"AvzConfig", "AvzBatchArgs", "AvzSpectralArgs"} <= set(shim)
    for name, fields in shim.items():
        assert fields == list(getattr(_lib, name)._fields_), name
