#!/usr/bin/env python3
"""Writes scenes/materials_lights.xml + .ecs: an open-topped room with one sphere per
reference material outside the BASELINE configs (Plastic, Dielectric, Mirror, Metal,
BrushedMetal, Velvet: devices/device_singleray/materials/*.h) lit by every analytic light
type (point, spot, directional, distant + a dim dome), for the SURVEY §8(f) rank-4 parity
tests. Deterministic; committed output."""
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent / "scenes"

MATS = [
    ("Plastic", [("float3", "pigmentColor", "0.8 0.1 0.1"), ("float", "roughness", "0.05")]),
    ("Plastic", [("float3", "pigmentColor", "0.1 0.6 0.1"), ("float", "roughness", "0")]),
    ("Dielectric", [("float", "etaInside", "1.5"), ("float3", "transmission", "0.9 0.95 0.99")]),
    ("Mirror", [("float3", "reflectance", "0.9 0.9 0.9")]),
    ("Metal", [("float3", "eta", "0.2 0.4 1.4"), ("float3", "k", "3.0 2.6 2.0"), ("float", "roughness", "0.1")]),
    ("Metal", [("float3", "reflectance", "0.95 0.8 0.6"), ("float", "roughness", "0")]),
    ("BrushedMetal", [("float3", "eta", "0.3 0.3 0.3"), ("float3", "k", "2.5 2.5 2.5"),
                      ("float", "roughnessX", "0.05"), ("float", "roughnessY", "0.4")]),
    ("Velvet", [("float3", "reflectance", "0.5 0.3 0.6"), ("float", "backScattering", "0.5"),
                ("float3", "horizonScatteringColor", "0.8 0.8 0.9"), ("float", "horizonScatteringFallOff", "2")]),
]


def material(code, parms):
    p = "".join(f'<{t} name="{n}">{v}</{t}>' for t, n, v in parms)
    return f'<material><code>"{code}"</code><parameters>{p}</parameters></material>'


def quad(a, b, c, d, mat):
    pos = " ".join(" ".join(map(str, v)) for v in (a, b, c, d))
    return (f"<TriangleMesh><positions>{pos}</positions><normals></normals><texcoords></texcoords>"
            f"<triangles>0 1 2 0 2 3</triangles>{mat}</TriangleMesh>")


def main():
    grey = material("Matte", [("float3", "reflectance", "0.5 0.5 0.5")])
    warm = material("Matte", [("float3", "reflectance", "0.6 0.5 0.4")])
    parts = [quad((560, 0, 0), (0, 0, 0), (0, 0, 560), (560, 0, 560), grey),            # floor
             quad((0, 0, 560), (0, 560, 560), (560, 560, 560), (560, 0, 560), warm),    # back wall
             quad((0, 0, 0), (0, 560, 0), (0, 560, 560), (0, 0, 560), grey)]            # left wall
    for i, (code, parms) in enumerate(MATS):
        x = 90 + (i % 4) * 127
        z = 170 + (i // 4) * 190
        parts.append(f"<Sphere><position>{x} 62 {z}</position><radius>60</radius><numTheta>24</numTheta>"
                     f"<numPhi>32</numPhi>{material(code, parms)}</Sphere>")
    # lights through the XML loader (xml_loader.cpp:274-324); the spot points down (-y)
    parts.append('<PointLight><AffineSpace translate="280 470 240"/><I>90000 90000 80000</I></PointLight>')
    parts.append("<SpotLight><AffineSpace>1 0 0 120  0 0 -1 520  0 1 0 430</AffineSpace><I>120000 100000 90000</I>"
                 "<angleMin>35</angleMin><angleMax>55</angleMax></SpotLight>")
    parts.append("<DistantLight><AffineSpace>1 0 0 0  0 0.6 -0.8 0  0 0.8 0.6 0</AffineSpace><L>1.8 1.6 1.3</L>"
                 "<halfAngle>6</halfAngle></DistantLight>")
    xml = '<?xml version="1.0"?>\n<scene>\n  <Group>\n    ' + "\n    ".join(parts) + "\n  </Group>\n</scene>\n"
    (ROOT / "materials_lights.xml").write_text(xml)
    (ROOT / "materials_lights.ecs").write_text(
        "-i materials_lights.xml\n-vp 280 480 -420 -vi 280 40 300 -vu 0 1 0 -fov 45\n"
        "-dirlight -1 -2 1 0.35 0.35 0.3\n-ambientlight 0.05 0.05 0.06\n"
        "-tMaxShadowRay 3000\n-renderer pathtracer { spp = 1 depth = 6 }\n")


if __name__ == "__main__":
    main()
