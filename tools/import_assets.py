"""Convert the reference's scene OBJ files into the package's bundled .npz assets.

Run in the container that has the read-only reference checkout:
    python tools/import_assets.py [/root/reference/assets]
The geometry is parsed by the native hrt_obj_load (load_obj semantics: one mesh per `o`, file
order, winding kept) and stored as float32 positions + uint32 indices per mesh, so the GPU box
(which has no /root/reference) renders exactly the triangles the OBJ files define.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from epq_raytracer_amd.scene import ASSET_DIR, load_obj, save_mesh_asset  # noqa: E402

SCENES = ("Cube", "box", "Cave", "island")


def main(src: str) -> None:
    os.makedirs(ASSET_DIR, exist_ok=True)
    for name in SCENES:
        meshes = load_obj(os.path.join(src, f"{name}.obj"))
        out = os.path.join(ASSET_DIR, f"{name}.npz")
        save_mesh_asset(meshes, out)
        print(f"{name}: {len(meshes)} meshes, {sum(m.indices.size // 3 for m in meshes)} triangles -> {out}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/assets")
