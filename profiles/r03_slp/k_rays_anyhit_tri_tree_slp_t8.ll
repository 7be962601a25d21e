  br i1 %1011, label %1188, label %1306

1188:                                             ; preds = %1187
  %1189 = load float, ptr addrspace(5) %951, align 8, !tbaa !14
  %1190 = load float, ptr addrspace(5) %952, align 4, !tbaa !14
  %1191 = load float, ptr addrspace(5) %953, align 8, !tbaa !14
  %1192 = load float, ptr addrspace(5) %971, align 4, !tbaa !14
  %1193 = load float, ptr addrspace(5) %972, align 8, !tbaa !14
  %1194 = load float, ptr addrspace(5) %973, align 4, !tbaa !14
  %1195 = load float, ptr addrspace(5) %949, align 8, !tbaa !47
  %1196 = load float, ptr addrspace(5) %950, align 4, !tbaa !50
  %1197 = shufflevector <4 x float> %1030, <4 x float> poison, <2 x i32> <i32 0, i32 3>
  %1198 = insertelement <2 x float> poison, float %1189, i32 0
  %1199 = shufflevector <2 x float> %1198, <2 x float> poison, <2 x i32> zeroinitializer
  %1200 = fsub <2 x float> %1197, %1199
  %1201 = shufflevector <4 x float> %1030, <4 x float> %1031, <2 x i32> <i32 1, i32 4>
  %1202 = insertelement <2 x float> poison, float %1190, i32 0
  %1203 = shufflevector <2 x float> %1202, <2 x float> poison, <2 x i32> zeroinitializer
  %1204 = fsub <2 x float> %1201, %1203
  %1205 = shufflevector <4 x float> %1030, <4 x float> %1031, <2 x i32> <i32 2, i32 5>
  %1206 = insertelement <2 x float> poison, float %1191, i32 0
  %1207 = shufflevector <2 x float> %1206, <2 x float> poison, <2 x i32> zeroinitializer
  %1208 = fsub <2 x float> %1205, %1207
  %1209 = shufflevector <4 x float> %1031, <4 x float> %1030, <2 x i32> <i32 2, i32 4>
  %1210 = shufflevector <4 x float> %1030, <4 x float> %1031, <2 x i32> <i32 3, i32 6>
  %1211 = fsub <2 x float> %1209, %1199
  %1212 = fsub <2 x float> %1210, %1199
  %1213 = shufflevector <4 x float> %1031, <4 x float> %1030, <2 x i32> <i32 3, i32 5>
  %1214 = shufflevector <4 x float> %1031, <4 x float> poison, <2 x i32> <i32 0, i32 3>
  %1215 = fsub <2 x float> %1213, %1203
  %1216 = fsub <2 x float> %1214, %1203
  %1217 = shufflevector <4 x float> %1032, <4 x float> %1030, <2 x i32> <i32 0, i32 6>
  %1218 = shufflevector <4 x float> %1031, <4 x float> %1032, <2 x i32> <i32 1, i32 4>
  %1219 = fsub <2 x float> %1217, %1207
  %1220 = fsub <2 x float> %1218, %1207
  %1221 = shufflevector <2 x float> %1200, <2 x float> %1211, <2 x i32> <i32 1, i32 2>
  %1222 = shufflevector <2 x float> %1204, <2 x float> %1215, <2 x i32> <i32 1, i32 2>
  switch i32 %986, label %1226 [
    i32 0, label %1223
    i32 1, label %1224
  ]

1223:                                             ; preds = %1188
  br label %1226

1224:                                             ; preds = %1188
  %1225 = shufflevector <2 x float> %1208, <2 x float> %1219, <2 x i32> <i32 1, i32 2>
  br label %1226

1226:                                             ; preds = %1224, %1223, %1188
  %1227 = phi <2 x float> [ %1211, %1223 ], [ %1215, %1224 ], [ %1219, %1188 ]
  %1228 = phi <2 x float> [ %1204, %1223 ], [ %1208, %1224 ], [ %1204, %1188 ]
  %1229 = phi <2 x float> [ %1200, %1223 ], [ %1204, %1224 ], [ %1208, %1188 ]
  %1230 = phi <2 x float> [ %1220, %1223 ], [ %1212, %1224 ], [ %1221, %1188 ]
  %1231 = phi <2 x float> [ %1216, %1223 ], [ %1225, %1224 ], [ %1222, %1188 ]
  %1232 = phi <2 x float> [ %1208, %1223 ], [ %1200, %1224 ], [ %1200, %1188 ]
  %1233 = insertelement <2 x float> poison, float %1192, i32 0
  %1234 = shufflevector <2 x float> %1233, <2 x float> poison, <2 x i32> zeroinitializer
  %1235 = fmul <2 x float> %1234, %1229
  %1236 = shufflevector <2 x float> %1229, <2 x float> %1227, <2 x i32> <i32 1, i32 2>
  %1237 = fmul <2 x float> %1234, %1236
  %1238 = insertelement <2 x float> poison, float %1193, i32 0
  %1239 = shufflevector <2 x float> %1238, <2 x float> poison, <2 x i32> zeroinitializer
  %1240 = fmul <2 x float> %1239, %1229
  %1241 = fmul <2 x float> %1239, %1236
  %1242 = fsub <2 x float> %1232, %1235
  %1243 = fsub <2 x float> %1230, %1237
  %1244 = fsub <2 x float> %1228, %1240
  %1245 = fsub <2 x float> %1231, %1241
  %1246 = extractelement <2 x float> %1245, i32 1
  %1247 = extractelement <2 x float> %1242, i32 0
  %1248 = fmul float %1246, %1247
  %1249 = extractelement <2 x float> %1244, i32 0
  %1250 = extractelement <2 x float> %1243, i32 1
  %1251 = fmul float %1249, %1250
  %1252 = fsub float %1248, %1251
  %1253 = fmul <2 x float> %1244, %1243
  %1254 = fmul <2 x float> %1245, %1242
  %1255 = fsub <2 x float> %1253, %1254
  %1256 = extractelement <2 x float> %1255, i32 1
  %1257 = fadd float %1256, %1252
  %1258 = extractelement <2 x float> %1255, i32 0
  %1259 = fadd float %1258, %1257
  %1260 = fcmp une float %1259, 0.000000e+00
  br i1 %1260, label %1261, label %1303

1261:                                             ; preds = %1226
  %1262 = fcmp oge float %1256, 0.000000e+00
  %1263 = fcmp oge float %1252, 0.000000e+00
  %1264 = and i1 %1262, %1263
  %1265 = fcmp oge float %1258, 0.000000e+00
  %1266 = and i1 %1265, %1264
  br i1 %1266, label %1273, label %1267

1267:                                             ; preds = %1261
  %1268 = fcmp ole float %1256, 0.000000e+00
  %1269 = fcmp ole float %1252, 0.000000e+00
  %1270 = and i1 %1268, %1269
  %1271 = fcmp ole float %1258, 0.000000e+00
  %1272 = and i1 %1271, %1270
  br i1 %1272, label %1273, label %1303

1273:                                             ; preds = %1267, %1261
  %1274 = bitcast float %1259 to i32
  %1275 = lshr i32 %1274, 23
  %1276 = and i32 %1275, 255
  %1277 = add nsw i32 %1276, -1
  %1278 = icmp ult i32 %1277, 252
  %1279 = tail call float @llvm.amdgcn.rcp.f32(float %1259)
  %1280 = fneg float %1259
  %1281 = tail call float @llvm.fma.f32(float %1280, float %1279, float 1.000000e+00)
  %1282 = tail call noundef float @llvm.fma.f32(float %1281, float %1279, float %1279)
  %1283 = fdiv float 1.000000e+00, %1259
  %1284 = select i1 %1278, float %1282, float %1283
  %1285 = insertelement <2 x float> poison, float %1194, i32 0
  %1286 = shufflevector <2 x float> %1285, <2 x float> poison, <2 x i32> zeroinitializer
  %1287 = fmul <2 x float> %1286, %1227
  %1288 = extractelement <2 x float> %1229, i32 1
  %1289 = fmul float %1194, %1288
  %1290 = fmul float %1289, %1252
  %1291 = fmul <2 x float> %1287, %1255
  %1292 = extractelement <2 x float> %1291, i32 1
  %1293 = fadd float %1292, %1290
  %1294 = extractelement <2 x float> %1291, i32 0
  %1295 = fadd float %1294, %1293
  %1296 = fmul float %1295, %1284
  %1297 = fcmp oge float %1296, 0.000000e+00
  %1298 = fcmp olt float %1296, %1196
  %1299 = and i1 %1297, %1298
  %1300 = fcmp ogt float %1296, %1195
  %1301 = and i1 %1300, %1299
  %1302 = select i1 %1301, i32 2, i32 0
  br label %1303

1303:                                             ; preds = %1273, %1267, %1226
  %1304 = phi i32 [ 0, %1267 ], [ 0, %1226 ], [ %1302, %1273 ]
  %1305 = icmp eq i32 %1304, 0
  br i1 %1305, label %1306, label %1712

1306:                                             ; preds = %1303, %1187
  %1307 = select i1 %993, i1 %1004, i1 false
  %1308 = icmp slt i32 %1003, -1
  %1309 = select i1 %1307, i1 %1308, i1 false
  br i1 %1309, label %1310, label %1712

1310:                                             ; preds = %1306
  store i32 %1003, ptr addrspace(5) %981, align 8, !tbaa !60
  store float %998, ptr addrspace(5) %982, align 4, !tbaa !61
  store i32 -1, ptr addrspace(5) %979, align 8, !tbaa !58
  br label %1712

1311:                                             ; preds = %984
  %1312 = icmp eq i32 %991, -1
  br i1 %1312, label %1313, label %1365

1313:                                             ; preds = %1311
  %1314 = icmp slt i32 %989, 0
  %1315 = load i32, ptr addrspace(5) %977, align 4
  %1316 = select i1 %1314, i32 0, i32 %1315
  %1317 = icmp eq i32 %990, %1316
  br i1 %1317, label %1318, label %1347

1318:                                             ; preds = %1313
  br i1 %1314, label %1365, label %1319

1319:                                             ; preds = %1318
