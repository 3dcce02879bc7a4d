"""Known answers pinning the renderer oracle (oracle/render_oracle.c): the restatement the GPU
renderer is checked against (tests/test_render_gpu.py) is itself checked here against closed-form
ray intersections of each primitive type and of a triangle mesh, the near-plane clip of
triangles, back-face culling, the nearest-hit rule, the camera pose from body and camera frames, and the shading
formula, on a synthetic scene (no GPU)."""

import numpy as np

from oracle import render as OR

W, H = 64, 48


def _scene(objects, cam_pos=(0.0, 0.0, 0.0), cam_quat=(1.0, 0.0, 0.0, 0.0), fovy=45.0, tris=None):
    """Minimal compiled-scene arrays: objects = [(type, size3, pos3, rgb3)], a world-body camera
    looking along -z; tris: [m, 3, 3] triangles of one mesh geom at the origin (type 7)."""
    n = len(objects) + (1 if tris is not None else 0)
    a = {"geom_type": np.zeros(n, np.int32), "geom_group": np.zeros(n, np.int32),
         "geom_ctype": np.full(n, -1, np.int32), "geom_csize": np.zeros((n, 3)), "geom_size": np.zeros((n, 3)),
         "geom_rgba": np.ones((n, 4)), "names_cam": np.array(["cam"]), "cam_body": np.array([0], np.int32),
         "cam_pos": np.array([cam_pos], np.float64), "cam_quat": np.array([cam_quat], np.float64),
         "cam_fovy": np.array([fovy]), "_znear": np.float64(0.01), "_extent": np.float64(2.0)}
    pos = np.zeros((n, 3))
    for g, (t, size, p, rgb) in enumerate(objects):
        a["geom_type"][g] = t
        a["geom_size"][g] = size
        a["geom_rgba"][g, :3] = rgb
        pos[g] = p
    if tris is not None:  # one mesh geom on the world body, its triangles in the body frame
        g = n - 1
        a["geom_type"][g] = 7
        a["geom_rgba"][g, :3] = (0.5, 0.5, 0.5)
        t = np.asarray(tris, np.float64)
        e1, e2 = t[:, 1] - t[:, 0], t[:, 2] - t[:, 0]
        nrm = np.cross(e1, e2)
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        packed = np.zeros((len(t), 16), np.float32)
        packed[:, 0:3], packed[:, 3:6], packed[:, 6:9], packed[:, 9:12] = t[:, 0], e1, e2, nrm
        packed[:, 12] = np.full(len(t), g, np.int32).view(np.float32)
        packed[:, 13:16] = (0.5, 0.5, 0.5)
        a["rmesh_body"] = np.array([0], np.int32)
        a["rmesh_geoms"] = np.array([g], np.int32)
        a["rmesh_tri_adr"] = np.array([0], np.int32)
        a["rmesh_tri_num"] = np.array([len(t)], np.int32)
        a["rmesh_tri"] = packed
    gxmat = np.tile(np.eye(3).reshape(1, 9), (n, 1))
    return a, pos, gxmat


def _cast(a, pos, gxmat, pix):
    prims = OR.scene_prims(a)
    return OR.cast(a, prims, pos, gxmat, np.zeros((1, 3)), np.array([[1.0, 0, 0, 0]]), "cam", W, H, pix)


CENTRE = np.array([[W / 2, H / 2]])


def test_centre_ray_depth_of_each_primitive():
    cases = [(2, (0.3, 0, 0), (0, 0, -2.0), 1.7),        # sphere: 2 - r
             (6, (0.2, 0.3, 0.4), (0, 0, -2.0), 1.6),    # box: 2 - half z
             (5, (0.25, 0.5, 0), (0, 0, -2.0), 1.5),     # cylinder along z: cap at 2 - h
             (3, (0.1, 0.4, 0), (0, 0, -2.0), 1.5),      # capsule along z: 2 - h - r
             (0, (0, 0, 0), (0, 0, -3.0), 3.0)]          # plane z = -3
    for t, size, p, want in cases:
        a, pos, gm = _scene([(t, size, p, (1, 1, 1))])
        g, d, _ = _cast(a, pos, gm, CENTRE)
        assert g[0] == 0, t
        np.testing.assert_allclose(d[0], want, rtol=0, atol=1e-12, err_msg=str(t))


def test_nearest_hit_wins_and_background():
    a, pos, gm = _scene([(2, (0.2, 0, 0), (0, 0, -3.0), (1, 0, 0)), (2, (0.2, 0, 0), (0, 0, -2.0), (0, 1, 0))])
    g, d, rgb = _cast(a, pos, gm, np.array([[W / 2, H / 2], [1.0, 1.0]]))
    assert g[0] == 1 and abs(d[0] - 1.8) < 1e-12
    assert g[1] == -1 and tuple(OR.to_u8(rgb[1])) == (230, 255, 255)  # background (0.9, 1, 1)


def test_shading_of_a_head_on_face():
    # box face towards the camera: n . v = 1, light along world -z gives n_z = +1 on that face
    a, pos, gm = _scene([(6, (0.2, 0.2, 0.2), (0, 0, -2.0), (0.5, 0.4, 0.2))])
    _, _, rgb = _cast(a, pos, gm, CENTRE)
    np.testing.assert_allclose(rgb[0], np.array([0.5, 0.4, 0.2]) * (0.1 + 0.6 + 0.3), atol=1e-12)


def test_triangles_hit_and_near_clip():
    # a square of two triangles at z = -1.5 facing the camera, and one 1 cm in front of the camera
    sq = [[[-0.5, -0.5, -1.5], [0.5, -0.5, -1.5], [0.5, 0.5, -1.5]], [[-0.5, -0.5, -1.5], [0.5, 0.5, -1.5], [-0.5, 0.5, -1.5]]]
    near = [[[-1, -1, -0.01], [1, -1, -0.01], [0, 1, -0.01]]]  # depth 0.01 < znear 0.02: clipped
    a, pos, gm = _scene([], tris=sq + near)
    g, d, _ = _cast(a, pos, gm, np.array([[W / 2 + 3.3, H / 2 - 2.1]]))
    assert g[0] == 0
    np.testing.assert_allclose(d[0], 1.5, atol=1e-12)


def test_back_faces_are_culled():
    # the same square wound clockwise as seen from the camera (its winding normal points away): not
    # drawn, as MuJoCo's default mjRND_CULL_FACE; the sphere behind it is seen through it
    sq = [[[-0.5, -0.5, -1.5], [0.5, 0.5, -1.5], [0.5, -0.5, -1.5]], [[-0.5, -0.5, -1.5], [-0.5, 0.5, -1.5], [0.5, 0.5, -1.5]]]
    a, pos, gm = _scene([(2, (0.2, 0, 0), (0, 0, -3.0), (1, 0, 0))], tris=sq)
    g, d, _ = _cast(a, pos, gm, CENTRE)
    assert g[0] == 0 and abs(d[0] - 2.8) < 1e-12
    a, pos, gm = _scene([(2, (0.2, 0, 0), (0, 0, -3.0), (1, 0, 0))], tris=[[t[0], t[2], t[1]] for t in sq])
    g, d, _ = _cast(a, pos, gm, CENTRE)
    assert g[0] == 1 and abs(d[0] - 1.5) < 1e-12  # wound counter-clockwise: the square


def test_camera_pose_from_the_camera_quaternion():
    # camera rotated 90 degrees about world x: it looks along world -y (a sphere placed there)
    c = np.cos(np.pi / 4)
    a, pos, gm = _scene([(2, (0.25, 0, 0), (0, 2.0, 0), (1, 1, 1))], cam_quat=(c, c, 0, 0))
    g, d, _ = _cast(a, pos, gm, CENTRE)
    assert g[0] == 0 and abs(d[0] - 1.75) < 1e-12


def test_off_axis_ray_direction():
    # pixel x at the right image edge: the ray's x slope is tan(fovy/2) * aspect
    a, pos, gm = _scene([(0, (0, 0, 0), (0, 0, -1.0), (1, 1, 1))])
    g, d, _ = _cast(a, pos, gm, np.array([[float(W), H / 2]]))
    assert g[0] == 0 and abs(d[0] - 1.0) < 1e-12  # depth is the camera-z distance, not the ray length


def test_body_frame_meshes_and_the_second_surface():
    # the mesh's body sits 1 m down the view axis, its square 0.5 m below the body origin: depth 1.5,
    # the triangle's geom id and colour; a sphere of another geom behind it is the second surface
    sq = [[[-0.5, -0.5, -0.5], [0.5, -0.5, -0.5], [0.5, 0.5, -0.5]], [[-0.5, -0.5, -0.5], [0.5, 0.5, -0.5], [-0.5, 0.5, -0.5]]]
    a, pos, gm = _scene([(2, (0.1, 0, 0), (0, 0, -2.5), (1, 0, 0))], tris=sq)
    a["rmesh_body"] = np.array([1], np.int32)  # body 1; the camera stays on the world body 0
    prims = OR.scene_prims(a)
    xpos = np.array([[0.0, 0.0, 0.0], [0.0, 0.0, -1.0]])
    xquat = np.array([[1.0, 0, 0, 0], [1.0, 0, 0, 0]])
    g, d, rgb, d2 = OR.cast(a, prims, pos, gm, xpos, xquat, "cam", W, H, CENTRE, second=True)
    assert g[0] == 1 and abs(d[0] - 1.5) < 1e-12 and abs(d2[0] - 2.4) < 1e-12
    np.testing.assert_allclose(rgb[0], np.full(3, 0.5 * (0.1 + 0.6 + 0.3)), atol=1e-7)


# ---- materials (round 6): textures, specular term, gradient skybox -----------------------------
TEX2 = np.array([[[255, 0, 0], [0, 255, 0]], [[0, 0, 255], [255, 255, 0]]], np.uint8)  # 2 x 2 RGB texels


def _with_materials(a, tex_type, spec=0.0, shin=0.5, rep=(1.0, 1.0), uniform=0.0, sky=((0.9, 1, 1), (0.9, 1, 1))):
    """Give every geom of a _scene the same material: the 2 x 2 texture TEX2 (2d or cube)."""
    n = len(a["geom_type"])
    a["geom_texid"] = np.zeros(n, np.int32)
    a["geom_matinfo"] = np.tile(np.array([spec, shin, rep[0], rep[1], uniform, 0.0], np.float32), (n, 1))
    a["tex_type"] = np.array([tex_type], np.int32)
    a["tex_size"] = np.array([[2, 2]], np.int32)
    a["tex_adr"] = np.array([0], np.int32)
    a["tex_rgb"] = TEX2.reshape(-1, 3)
    a["sky_rgb"] = np.array(sky, np.float64)
    return a


def _pixel_of(point):
    """Continuous pixel coordinates of a camera-frame point (the camera at the origin, looking along
    -z, fovy 45 degrees, W x H)."""
    t = np.tan(np.deg2rad(22.5))
    x, y, z = point
    return np.array([[(x / -z / (t * W / H) + 1.0) * W / 2, (1.0 - y / -z / t) * H / 2]])


def _shade(point):
    """0.1 + 0.6 n.v + 0.3 n.z of a face with n = +z seen from the origin at camera-frame `point`."""
    return 0.1 + 0.6 * (-point[2] / np.linalg.norm(point)) + 0.3


def test_2d_texture_on_a_plane_texel_centres_and_repeat():
    # an infinite plane 3 m down, texuniform: one period per metre; texel (col, row) centred at
    # ((col + 0.5) / 2, (row + 0.5) / 2) of the period, wrapped every metre
    a, pos, gm = _scene([(0, (0, 0, 0), (0, 0, -3.0), (1, 1, 1))])
    _with_materials(a, 0, uniform=1.0)
    for (x, y), (row, col) in [((0.25, 0.25), (0, 0)), ((0.75, 0.25), (0, 1)), ((0.25, 0.75), (1, 0)),
                               ((-0.25, -0.25), (1, 1)), ((1.75, 0.25), (0, 1))]:
        _, _, rgb = _cast(a, pos, gm, _pixel_of((x, y, -3.0)))
        np.testing.assert_allclose(rgb[0], TEX2[row, col] / 255.0 * _shade((x, y, -3.0)), atol=1e-9,
                                   err_msg=str((x, y)))
    # between texel centres: the bilinear blend of the four (wrapped) neighbours
    _, _, rgb = _cast(a, pos, gm, _pixel_of((0.5, 0.5, -3.0)))
    np.testing.assert_allclose(rgb[0], TEX2.reshape(-1, 3).mean(0) / 255.0 * _shade((0.5, 0.5, -3.0)), atol=1e-9)


def test_2d_texture_repeated_over_a_finite_plane():
    # plane half extents (1, 1), texrepeat (2, 2), not uniform: the image repeats twice over 2 m
    a, pos, gm = _scene([(0, (1.0, 1.0, 0), (0, 0, -3.0), (1, 1, 1))])
    _with_materials(a, 0, rep=(2.0, 2.0))
    # u = 2 (x / 2 + 0.5): x = -0.75 -> u = 0.25 (texel column 0), x = -0.25 -> 0.75 (column 1),
    # x = 0.25 -> 1.25 (column 0 of the second repeat)
    for x, col in ((-0.75, 0), (-0.25, 1), (0.25, 0)):
        _, _, rgb = _cast(a, pos, gm, _pixel_of((x, -0.75, -3.0)))
        np.testing.assert_allclose(rgb[0], TEX2[0, col] / 255.0 * _shade((x, -0.75, -3.0)), atol=1e-9, err_msg=str(x))


def test_cube_texture_on_a_box_face():
    # a 0.8 m cube 2 m down the view axis, cube texture in metric coordinates: its +z face centre
    # looks up the middle of the face image (the four texels' mean), (0.2, 0.2, 0.4) looks up
    # s = 0.75, t = 0.25: texel (col 1, row 0) exactly
    a, pos, gm = _scene([(6, (0.4, 0.4, 0.4), (0, 0, -2.4), (1, 1, 1))])
    _with_materials(a, 1)
    _, _, rgb = _cast(a, pos, gm, CENTRE)
    np.testing.assert_allclose(rgb[0], TEX2.reshape(-1, 3).mean(0) / 255.0, atol=1e-9)
    _, _, rgb = _cast(a, pos, gm, _pixel_of((0.2, 0.2, -2.0)))
    np.testing.assert_allclose(rgb[0], TEX2[0, 1] / 255.0 * _shade((0.2, 0.2, -2.0)), atol=1e-9)


def test_specular_highlight_of_a_face_under_the_light():
    # camera looking down world -z at a face whose normal points at it and at the light: n.h = 1,
    # so the specular term is specular x 0.3 whatever the shininess
    a, pos, gm = _scene([(6, (0.2, 0.2, 0.2), (0, 0, -2.0), (0.5, 0.4, 0.2))])
    _with_materials(a, 0, spec=0.5, shin=0.7)
    a["geom_texid"][:] = -1
    _, _, rgb = _cast(a, pos, gm, CENTRE)
    np.testing.assert_allclose(rgb[0], np.array([0.5, 0.4, 0.2]) * 1.0 + 0.5 * 0.3, atol=1e-12)
    # off-centre on the same face: n.h = cos of half the view angle, raised to 128 x shininess
    pix = _pixel_of((0.1, 0.0, -1.8))
    _, _, rgb2 = _cast(a, pos, gm, pix)
    v = np.array([-0.1, 0.0, 1.8]) / np.linalg.norm([0.1, 0.0, 1.8])
    h = (v + np.array([0, 0, 1.0])) / np.linalg.norm(v + np.array([0, 0, 1.0]))
    want = np.array([0.5, 0.4, 0.2]) * (0.1 + 0.6 * v[2] + 0.3) + 0.5 * 0.3 * h[2] ** (128 * 0.7)
    np.testing.assert_allclose(rgb2[0], want, atol=1e-12)


def test_gradient_skybox_behind_everything():
    a, pos, gm = _scene([(2, (0.1, 0, 0), (5.0, 5.0, -3.0), (1, 1, 1))])
    _with_materials(a, 0, sky=((0.2, 0.4, 0.6), (0.8, 0.6, 0.4)))
    g, _, rgb = _cast(a, pos, gm, CENTRE)  # straight down world -z: rgb2
    assert g[0] == -1
    np.testing.assert_allclose(rgb[0], [0.8, 0.6, 0.4], atol=1e-12)
    c = np.cos(np.pi / 4)
    a, pos, gm = _scene([(2, (0.1, 0, 0), (5.0, 5.0, -3.0), (1, 1, 1))], cam_quat=(c, c, 0, 0))
    _with_materials(a, 0, sky=((0.2, 0.4, 0.6), (0.8, 0.6, 0.4)))
    _, _, rgb = _cast(a, pos, gm, CENTRE)  # horizontal: halfway
    np.testing.assert_allclose(rgb[0], [0.5, 0.5, 0.5], atol=1e-12)


def test_mip_level_from_the_pixel_footprint():
    # a 4 x 4 texture, one period per metre, on a plane facing the camera at the distance where one
    # pixel step of the centre ray spans exactly 2 texels: level of detail 1, the level-1 texel
    # (the rounded mean of its 2 x 2 block) at its centre, no blend with another level; at a tenth of
    # that distance the footprint is below a texel: level 0, bilinear
    tex = np.arange(48, dtype=np.uint8).reshape(4, 4, 3) * 5
    step = 2 * np.tan(np.deg2rad(22.5)) / H  # one pixel's step of the ray slope (square pixels)
    d = 2.0 / (4 * step)
    a, pos, gm = _scene([(0, (0, 0, 0), (-0.25, -0.25, -d), (1, 1, 1))])
    _with_materials(a, 0, uniform=1.0)
    a["tex_size"] = np.array([[4, 4]], np.int32)
    a["tex_rgb"] = tex.reshape(-1, 3)
    _, _, rgb = _cast(a, pos, gm, CENTRE)
    lvl1 = (tex[0, 0].astype(int) + tex[0, 1] + tex[1, 0] + tex[1, 1] + 2) // 4
    np.testing.assert_allclose(rgb[0], lvl1 / 255.0, atol=1e-9)
    a, pos, gm = _scene([(0, (0, 0, 0), (-0.25 + 1 / 8, -0.25 + 1 / 8, -d / 10), (1, 1, 1))])
    _with_materials(a, 0, uniform=1.0)
    a["tex_size"] = np.array([[4, 4]], np.int32)
    a["tex_rgb"] = tex.reshape(-1, 3)
    _, _, rgb = _cast(a, pos, gm, CENTRE)  # local (1/8, 1/8): texel (0, 0)'s centre of level 0
    np.testing.assert_allclose(rgb[0], tex[0, 0] / 255.0, atol=1e-9)
