"""Gmsh 2.2 binary reader (spectralelementmethod_amd.grid_importers) against
what the REFERENCE reader (sem/grid_importers.py:45-68, run by
tests/golden/make_goldens.py gen_msh) built from the same committed .msh
files: nodes, lexicographic cell node maps, regions, cell adjacency and
boundary sides -- plus writer round trips and the reference's error
behaviour.  CPU only."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

CASES = ["sq_p4", "sq_p2", "sq_p8"]


@pytest.fixture(scope="module")
def ref():
    return load_golden("msh_reference.npz")


def _boundary_rows(mesh):
    rows = []
    for cell in sorted(mesh._boundary_map):
        for bid in sorted(mesh._boundary_map[cell]):
            for k, bd in enumerate(mesh._boundary_map[cell][bid]):
                rows.append((cell, bid, k, bd.ndim, bd.index))
    return np.array(rows, dtype=np.int64)


@pytest.mark.parametrize("name", CASES)
def test_load_msh_matches_reference_reader(ref, name):
    from spectralelementmethod_amd import grid_importers as gi
    mesh = gi.load_msh(os.path.join(GOLDEN, "mesh_%s.msh" % name), 2)
    assert np.array_equal(mesh.nodes, ref[name + "_nodes"])
    assert np.array_equal(mesh.element_map(), ref[name + "_e2n"])
    assert np.array_equal(np.array(mesh._region_ids), ref[name + "_region"])
    assert list(mesh._region_names) == list(ref[name + "_region_names"])
    assert list(mesh._boundary_names) == list(ref[name + "_boundary_names"])
    assert np.array_equal(mesh._adj, ref[name + "_adj"])
    assert np.array_equal(_boundary_rows(mesh), ref[name + "_bnd"])
    # cells expose the reference's per-cell views
    cell = mesh.get_cell(0)
    assert cell.region_name == "interior"
    assert [a if a is not None else -1 for a in cell._adj_map] == list(ref[name + "_adj"][0])
    assert sorted(mesh._boundary_cells[0]) == sorted(set(ref[name + "_bnd"][ref[name + "_bnd"][:, 1] == 0, 0]))


@pytest.mark.parametrize("p", [1, 2, 3, 5, 7, 10])
def test_write_load_round_trip(tmp_path, p):
    from spectralelementmethod_amd import grid_importers as gi, meshgen
    path = str(tmp_path / "m.msh")
    nodes, e2n = meshgen.write_square_msh(path, 4, 3, p, warp=0.05 if p > 1 else 0.0)
    mesh = gi.load_msh(path, 2)
    assert np.array_equal(mesh.nodes, nodes)
    assert np.array_equal(mesh.element_map(), e2n)
    assert mesh.n_boundary_cells == 2 * (4 + 3) - 4  # perimeter cells
    names = list(mesh._boundary_names)
    assert [len(mesh._boundary_cells[names.index(b)]) for b in ("ebc", "nbc")] == [6, 6]


def test_gmsh_order_is_the_inverse_of_the_reader():
    from spectralelementmethod_amd.grid_importers import gmsh_to_lexicographic
    for shape in [(2, 2), (3, 3), (5, 5), (11, 11), (4,), (9,)]:
        idx = gmsh_to_lexicographic(shape).ravel()
        assert sorted(idx.tolist()) == list(range(int(np.prod(shape))))
    # Gmsh numbering of a 9-node quadrilateral: vertices ccw, edge midpoints, centre
    assert gmsh_to_lexicographic((3, 3)).tolist() == [[0, 7, 3], [4, 8, 6], [1, 5, 2]]


def test_format_errors(tmp_path):
    from spectralelementmethod_amd import grid_importers as gi
    good = open(os.path.join(GOLDEN, "mesh_sq_p2.msh"), "rb").read()
    cases = {"version": good.replace(b"2.2 1 8", b"4.1 1 8", 1),
             "datasize": good.replace(b"2.2 1 8", b"2.2 1 4", 1),
             "header": b"$Mesh" + good[12:],
             "truncated": good[:len(good) // 2]}
    for key, blob in cases.items():
        path = str(tmp_path / (key + ".msh"))
        open(path, "wb").write(blob)
        with pytest.raises(gi.FileFormatError):
            gi.load_msh(path, 2)
    path = str(tmp_path / "ascii.msh")
    open(path, "wb").write(b"$MeshFormat\n2.2 0 8\n$EndMeshFormat\n")
    with pytest.raises(NotImplementedError):
        gi.load_msh(path, 2)
